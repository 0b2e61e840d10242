// gaussian_tables.h — the denoiser's precomputed Gaussian weights, gaussian.cuh:12-43
// (USE_PRECALCULATED_GAUSSIAN 1, gaussian.cuh:8): the reference's literals, each converted to
// float once as its float arrays do.  One list for the device tables (denoise.hip __constant__)
// and the host copy rt_filter_kernel hands out, so both are the same values.
#pragma once

#define RT_GAUSS3_INIT                                                                                    \
    {(float)0.0578968, (float)0.0921378, (float)0.0584323, (float)0.0921378, (float)0.146629,                \
     (float)0.09299,   (float)0.0584322, (float)0.0929898, (float)0.0589727}

#define RT_GAUSS5_INIT                                                                                    \
    {(float)0.00360466, (float)0.0144464, (float)0.0229902, (float)0.01458,   (float)0.0036719,              \
     (float)0.0144464,  (float)0.0578968, (float)0.0921378, (float)0.0584323, (float)0.0147159,              \
     (float)0.0229902,  (float)0.0921378, (float)0.146629,  (float)0.09299,   (float)0.023419,               \
     (float)0.01458,    (float)0.0584322, (float)0.0929898, (float)0.0589727, (float)0.014852,               \
     (float)0.00367191, (float)0.0147158, (float)0.0234191, (float)0.0148519, (float)0.0037404}

#define RT_GAUSS7_INIT                                                                                    \
    {(float)3.47404e-05, (float)0.000353875, (float)0.00141822, (float)0.00225698, (float)0.00143134,         \
     (float)0.000360475, (float)3.57221e-05, (float)0.000353875, (float)0.00360466, (float)0.0144464,         \
     (float)0.0229902,   (float)0.01458,     (float)0.0036719,  (float)0.000363875, (float)0.00141822,        \
     (float)0.0144464,   (float)0.0578968,   (float)0.0921378,  (float)0.0584323,  (float)0.0147159,          \
     (float)0.0014583,   (float)0.00225698,  (float)0.0229902,  (float)0.0921378,  (float)0.146629,           \
     (float)0.09299,     (float)0.023419,    (float)0.00232076, (float)0.00143134, (float)0.01458,            \
     (float)0.0584322,   (float)0.0929898,   (float)0.0589727,  (float)0.014852,   (float)0.00147179,         \
     (float)0.000360475, (float)0.00367191,  (float)0.0147158,  (float)0.0234191,  (float)0.0148519,          \
     (float)0.0037404,   (float)0.000370662, (float)3.57221e-05, (float)0.000363875, (float)0.0014583,        \
     (float)0.00232075,  (float)0.00147179,  (float)0.000370662, (float)3.67315e-05}
