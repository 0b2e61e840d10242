#!/usr/bin/env python3
"""Per-kernel summary of separate rocprofv3 --pmc passes (tools/prof.sh).

    python tools/pmc_report.py <out.json> <pass_dir>... [--key KEY] [--workload TEXT] [--calib FILE]
    python tools/pmc_report.py --make-calib <calib.json> <fetch_pass_dir> <write_pass_dir>

--make-calib reads the FETCH_SIZE and WRITE_SIZE passes of tools/probe/fetch_calib.bin (streaming
copies of 4, 8 and 16 bytes per lane and a 16x16-tiled 8-byte half4 copy, each of a known byte
count) and writes, per access width, the factor that turns FETCH_SIZE x 1024 into the bytes read.
--calib applies those factors: the denoise / post kernels (8-byte half4 texel reads) take the
8-byte factor, every other kernel the 16-byte one (MI355X_MICROARCH.md: 2, FETCH_SIZE counts half
the bytes of 16-byte-per-lane reads).  Without --calib every kernel takes 2.

Kernels are named by their symbol with boolean template arguments dropped and integer ones kept
(k_spatial5<3, false> -> k_spatial5<3>, k_temporal<true> -> k_temporal; k_scale_post<576> ->
k_scale_post); k_build_bvh<threads> is labelled by its workgroup count (k_build_bvh@61wg, @938wg).  Per kernel the median per-dispatch value of every
counter is taken, then (MI355X_MICROARCH.md HBM, L2 and SQ sections):
  hbm_bytes          = (f * FETCH_SIZE + WRITE_SIZE) * 1024   (FETCH_SIZE, KB, counts half the bytes
                       of wide reads on gfx950: f = 2, or the calibrated factor of the kernel's
                       access width, --calib; WRITE_SIZE in KB)
  l2_hit_rate        = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  valu_busy_frac     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  wait_inst_any_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls)
  wait_any_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / barriers)
  valu_per_wave, lds_per_wave = SQ_INSTS_VALU, SQ_INSTS_LDS per wave
  us                 = the dispatch's duration (median over the passes' dispatches)
The path-trace stage's HBM bytes (`stage_hbm_bytes`, the seven kernels bench.py names) and the
denoise/post chain's (`denoise_hbm_bytes`) are sums of per-kernel medians."""
import collections
import csv
import glob
import json
import re
import statistics
import sys

STAGE = ("k_pt_camera", "k_pt_shade0", "k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>",
         "k_pt_resume<4>", "k_pt_resolve")
DENOISE = ("k_temporal", "k_spatial7", "k_spatial5<3>", "k_spatial5<6>", "k_spatial5<12>", "k_temporal2",
           "k_downscale_chain", "k_scale_post")


def short(name, grid, wg):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    n = re.sub(r"<(\d+)(, (true|false))+>", r"<\1>", n)
    n = re.sub(r"<(true|false)(, (true|false))*>", "", n)
    n = re.sub(r"^k_scale_post<\d+>$", "k_scale_post", n)  # its LDS tile size (24 x 24 or 48 x 48)
    if n.startswith("k_build_bvh") and wg:
        n = "k_build_bvh@%dwg" % (grid // wg)
    return n


# a denoise pass's kernel when the frame runs the active-tile-list chain (bench.py PMC_LIST_NAMES)
LIST_NAMES = {"k_spatial7": ("k_spatial7_list2", "k_spatial7_list"), "k_spatial5<3>": ("k_spatial5_list2<3>", "k_spatial5_list<3>"),
              "k_spatial5<6>": ("k_spatial5_list2<6>", "k_spatial5_list<6>"), "k_spatial5<12>": ("k_spatial5_list2<12>",)}

# kernels whose reads are 8-byte half4 texels (the denoiser and the post chain)
HALF4_KERNELS = set(DENOISE) | {"k_spatial7_list", "k_spatial5_list<3>", "k_spatial5_list<6>", "k_spatial7_list2",
                                "k_spatial5_list2<3>", "k_spatial5_list2<6>", "k_spatial5_list2<12>", "k_tile_noise",
                                "k_noise16", "k_downscale4", "k_histogram", "k_bloom_gauss", "k_bloom_apply",
                                "k_lens_flare", "k_hdr_out"}
# tools/probe/fetch_calib.hip: bytes each way per dispatch
CALIB_BYTES = {"copy_k<unsigned int>": (4, 512 << 20), "copy_k<HIP_vector_type<unsigned int, 2u> >": (8, 512 << 20),
               "copy_k<HIP_vector_type<unsigned int, 4u> >": (16, 512 << 20), "tile8_k": ("tile8", 1920 * 1080 * 8)}


def counters_per_kernel(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("void ", "").split("(")[0]
        for did, v in per.items():
            out[names[did]].append(v)
    return out


def make_calib(out_path, fetch_dir, write_dir):
    fetch, write = counters_per_kernel(fetch_dir, "FETCH_SIZE"), counters_per_kernel(write_dir, "WRITE_SIZE")
    res = {"source": "tools/probe/fetch_calib.bin: FETCH_SIZE and WRITE_SIZE passes (rocprofv3 --pmc, one each)",
           "widths": {}}
    for name, (width, nbytes) in CALIB_BYTES.items():
        if name not in fetch or name not in write:
            continue
        fk, wk = statistics.median(fetch[name]), statistics.median(write[name])
        res["widths"][str(width)] = {"kernel": name, "bytes_each_way": nbytes, "dispatches": len(fetch[name]),
                                     "fetch_size_kb": fk, "write_size_kb": wk,
                                     "fetch_factor": round(nbytes / (fk * 1024.0), 4),
                                     "write_factor": round(nbytes / (wk * 1024.0), 4)}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for w, e in res["widths"].items():
        print("%-6s fetch x%.3f write x%.3f  (%s)" % (w, e["fetch_factor"], e["write_factor"], e["kernel"]))


def main():
    args = sys.argv[1:]
    if args and args[0] == "--make-calib":
        make_calib(*args[1:4])
        return
    calib = None
    if "--calib" in args:
        i = args.index("--calib")
        calib = json.load(open(args[i + 1]))["widths"]
        del args[i:i + 2]
    key = workload = None
    if "--key" in args:
        i = args.index("--key")
        key = args[i + 1]
        del args[i:i + 2]
    if "--workload" in args:
        i = args.index("--workload")
        workload = args[i + 1]
        del args[i:i + 2]
    out_path, dirs = args[0], args[1:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            span = {}
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"], int(r["Grid_Size"] or 0), int(r["Workgroup_Size"] or 0))
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                span[(k, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for (k, did), c in per.items():
                for n, v in c.items():
                    vals[k][n].append(v)
                dur[k].append(span[(k, did)])
    kernels = {}
    for k, cv in vals.items():
        c = {n: statistics.median(v) for n, v in cv.items()}
        e = {"dispatches": max(len(v) for v in cv.values()), "us": round(statistics.median(dur[k]), 2)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fac = 2.0
            if calib:
                fac = calib["8" if k in HALF4_KERNELS else "16"]["fetch_factor"]
            e["fetch_factor"] = fac
            e["hbm_bytes"] = int(round((fac * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024))
            e["fetch_bytes"] = int(round(fac * c["FETCH_SIZE"] * 1024))
            e["write_bytes"] = int(round(c["WRITE_SIZE"] * 1024))
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = round(hit / (hit + miss), 4)
        wc, w = c.get("SQ_WAVE_CYCLES"), c.get("SQ_WAVES")
        if wc:
            for n, f in (("SQ_ACTIVE_INST_VALU", "valu_busy_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                         ("SQ_WAIT_ANY", "wait_any_frac")):
                if n in c:
                    e[f] = round(c[n] / wc, 4)
        if w:
            e["waves"] = int(w)
            for n, f in (("SQ_INSTS_VALU", "valu_per_wave"), ("SQ_INSTS_LDS", "lds_per_wave")):
                if n in c:
                    e[f] = round(c[n] / w, 1)
        e["counters_median"] = c
        kernels[k] = e
    res = {"workload_key": key, "workload": workload, "passes": dirs, "kernels": kernels,
           "stage_hbm_bytes": sum(kernels[k].get("hbm_bytes", 0) for k in STAGE if k in kernels) or None,
           "denoise_hbm_bytes": sum(kernels[k].get("hbm_bytes", 0) for k in
                                    (next((n for n in LIST_NAMES.get(d, ()) + (d,) if n in kernels), None)
                                     for d in DENOISE) if k) or None,
           "correction": ("FETCH_SIZE x the calibrated factor of the kernel's access width (--calib: 8-byte half4 "
                          "reads for the denoise / post kernels, 16-byte otherwise), KB x 1024" if calib else
                          "FETCH_SIZE doubled (gfx950 counts half the bytes of wide reads), KB x 1024"),
           "note": "every counter group from its own rocprofv3 --pmc run; medians over all dispatches of the kernel"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    order = sorted(kernels, key=lambda k: -kernels[k]["us"] * kernels[k]["dispatches"])
    for k in order:
        e = kernels[k]
        print("%-22s n=%4d %9.2f us %s" % (k[:22], e["dispatches"], e["us"], " ".join(
            "%s=%s" % (f, e[f]) for f in ("hbm_bytes", "l2_hit_rate", "valu_busy_frac", "wait_inst_any_frac",
                                          "wait_any_frac", "waves", "valu_per_wave", "lds_per_wave") if f in e)))


if __name__ == "__main__":
    main()
