"""HBM traffic per kernel launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/gpu_round.sh (one pass per counter), corrected as MI355X_MICROARCH.md prescribes for gfx950:
FETCH_SIZE counts half of the bytes of WIDE STREAMING reads (16 B per lane) -- doubled only for the
kernels whose reads are of that kind (the shuffle / unshuffle filters); the LZ encoder and decoder
read with dword and scattered loads, whose FETCH_SIZE is uncalibrated, so they are reported raw
with the doubled figure beside it as an upper bound.  WRITE_SIZE is exact; both are in KiB.
    python tools/pmc_traffic.py <gpurun_out dir> <tag> <out.json> [exact|fast] [workload]"""
import collections
import csv
import json
import os
import sys

WORKLOAD = "T: float32 ts=4 SHUFFLE+BloscLZ clevel 5, 256 KiB blocks, 4 MiB chunks x 1024 per GPU"
STREAMING = ("k_ffilter", "k_dfilter", "k_copy16")


def main(root, tag, dst, mode="fast", workload=WORKLOAD):
    kern = collections.defaultdict(dict)
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(root, f"pmc_{tag}_{ctr}", "run_counter_collection.csv"))):
            vals[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            kern[k][ctr + "_KiB_per_launch"] = sum(v) / len(v)
            kern[k]["launches"] = len(v)
    for k, v in kern.items():
        f = v.get("FETCH_SIZE_KiB_per_launch", 0.0) * 1024
        w = v.get("WRITE_SIZE_KiB_per_launch", 0.0) * 1024
        streaming = k.split("<")[0].split("::")[-1] in STREAMING
        v["hbm_bytes_per_launch"] = (2 * f if streaming else f) + w
        v["hbm_bytes_upper_bound"] = 2 * f + w
        v["correction"] = ("2 x FETCH + WRITE (16 B/lane streaming reads)" if streaming else
                           "FETCH + WRITE raw (dword / scattered reads: FETCH_SIZE uncalibrated; "
                           "hbm_bytes_upper_bound doubles FETCH)")
    res = {"workload": workload + f" [{mode}]", "tag": tag,
           "command": "rocprofv3 --pmc <FETCH_SIZE|WRITE_SIZE> --kernel-include-regex ... -- " +
                      (f"python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lz-mode {mode}" if workload == WORKLOAD
                       else f"python3 tools/bench_configs.py --only <cfg> --lz-mode {mode} --steps 1") + " (one pass per counter)",
           "kernels": kern}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
