# Build recipe (no cmake in the product path).  `make -j8` builds:
#   real-time-ray-tracing_amd/lib/librtx.so   the product: HIP kernels for gfx950 + host runtime + C-ABI
#   oracle/_build/liboracle.so                the CPU restatement (test infrastructure only)
#   oracle/_build/liboracle_libm.so           the same with host-libm transcendentals (parity metric)
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
PKG      := real-time-ray-tracing_amd
CSRC     := $(PKG)/csrc
LIBDIR   := $(PKG)/lib
OBJDIR   := $(PKG)/lib/obj
# -ffp-contract=off on host AND device: every expression rounds once per operation, as the
# CPU oracle does (DESIGN.md §4 numerics policy).
HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -I$(CSRC) $(ABLFLAGS)
CXXFLAGS := -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude -I$(CSRC)

HIP_SRCS := $(wildcard $(CSRC)/*.hip)
CPP_SRCS := $(wildcard $(CSRC)/*.cpp)
HDRS     := $(wildcard $(CSRC)/*.h) include/rtx_amd.h
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.hip.o,$(HIP_SRCS))
CPP_OBJS := $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.cpp.o,$(CPP_SRCS))

ORC_SRCS := $(wildcard oracle/*.cpp)
ORC_HDRS := $(wildcard oracle/*.h) $(CSRC)/rtmath.h $(CSRC)/soil_textures.h

all: $(LIBDIR)/librtx.so $(LIBDIR)/librtx_rccl.so oracle/_build/liboracle.so oracle/_build/liboracle_libm.so \
     oracle/_build/liboracle_libm_fma.so

$(OBJDIR)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(filter-out --offload-arch=gfx950,$(HIPFLAGS)) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -x c++ -c $< -o $@

$(LIBDIR)/librtx.so: $(HIP_OBJS) $(CPP_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $^ -ldl

# the RCCL communicator of include/rtx_dist.h, separate so that librtx.so does not need librccl
$(LIBDIR)/librtx_rccl.so: $(CSRC)/rccl/dist_rccl.cpp include/rtx_dist_rccl.h include/rtx_dist.h $(LIBDIR)/librtx.so
	$(HIPCC) $(filter-out --offload-arch=gfx950,$(HIPFLAGS)) -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -x c++ -shared \
	    -o $@ $< -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle/_build/liboracle.so: $(ORC_SRCS) $(ORC_HDRS) $(CSRC)/soil_textures.cpp
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -shared -o $@ $(ORC_SRCS) $(CSRC)/soil_textures.cpp -lpthread

# the same restatement with host-libm transcendentals (parity metric, ocommon.h ORC_LIBM)
oracle/_build/liboracle_libm.so: $(ORC_SRCS) $(ORC_HDRS) $(CSRC)/soil_textures.cpp
	@mkdir -p oracle/_build
	$(CXX) $(CXXFLAGS) -DORC_LIBM -shared -o $@ $(ORC_SRCS) $(CSRC)/soil_textures.cpp -lpthread

# ... and with nvcc's default contraction (the reference builds with CMake's nvcc defaults,
# CMakeLists.txt:42, no --fmad=false): every a*b+c the compiler finds becomes one fused multiply-add,
# in the restatement of the reference's device code.  The procedural scene and the soil textures
# are host code in the reference (terrain.cpp) and inputs here, so they stay uncontracted.
ORC_FMA_DEV  := $(filter-out oracle/scene.cpp,$(ORC_SRCS))
ORC_FMA_OBJS := $(patsubst oracle/%.cpp,oracle/_build/fma/%.o,$(ORC_FMA_DEV))
oracle/_build/fma/%.o: oracle/%.cpp $(ORC_HDRS)
	@mkdir -p oracle/_build/fma
	$(CXX) $(filter-out -ffp-contract=off,$(CXXFLAGS)) -ffp-contract=fast -mfma -DORC_LIBM -c $< -o $@
oracle/_build/fma/scene.o: oracle/scene.cpp $(ORC_HDRS)
	@mkdir -p oracle/_build/fma
	$(CXX) $(CXXFLAGS) -DORC_LIBM -c $< -o $@
oracle/_build/fma/soil_textures.o: $(CSRC)/soil_textures.cpp $(ORC_HDRS)
	@mkdir -p oracle/_build/fma
	$(CXX) $(CXXFLAGS) -DORC_LIBM -c $< -o $@
oracle/_build/liboracle_libm_fma.so: $(ORC_FMA_OBJS) oracle/_build/fma/scene.o oracle/_build/fma/soil_textures.o
	$(CXX) -shared -o $@ $^ -lpthread

clean:
	rm -rf $(LIBDIR) oracle/_build

.PHONY: all clean
