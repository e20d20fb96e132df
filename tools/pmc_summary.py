"""Summarise the rocprofv3 --pmc passes of tools/run_pmc.sh for the integrate kernel.

usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<name>_pmc.json [kernel] [workload text] [rays]
Counter values are summed over the rows of each dispatch of grt::integrate_kernel<1>
(one C2 frame per dispatch) and reported per launch.  FETCH_SIZE (KB) is doubled per
the gfx950 correction in MI355X_MICROARCH.md; WRITE_SIZE (KB) is taken as is.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gr_raytracer_amd._lib import device_code_sha256, kernel_code_sha256, kernel_symbol  # noqa: E402

KERNEL = sys.argv[3] if len(sys.argv) > 3 else "grt::integrate_kernel<1, false>"
WORKLOAD = sys.argv[4] if len(sys.argv) > 4 else "one frame of tools/prof_target.py c2 (1500x1500, 2.25M rays)"
RAYS = int(sys.argv[5]) if len(sys.argv) > 5 else 2250000  # rays per launch of the profiled workload


def load(pass_dir):
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    dur = {}
    for f in glob.glob(str(Path(pass_dir) / "**" / "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                d = row["Dispatch_Id"]
                vals[row["Counter_Name"]][d] += float(row["Counter_Value"])
                dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return vals, dur


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    counters, kernel_ms = {}, {}
    for p in ("fetch", "write", "valu", "busy", "mem"):
        if not (src / p).exists():
            continue
        vals, dur = load(src / p)
        for c, per in vals.items():
            counters[c] = sum(per.values()) / len(per)
        if dur:
            kernel_ms[p] = sum(dur.values()) / len(dur)
    fetch_b = counters.get("FETCH_SIZE", 0.0) * 1024 * 2
    write_b = counters.get("WRITE_SIZE", 0.0) * 1024
    out = {
        "kernel": f"{KERNEL}, {WORKLOAD}",
        "rays_per_launch": RAYS,  # bench.py uses the traffic only for a launch of this size
        # the device code the passes measured: bench.py refuses a summary of another build
        "code_object_sha256": device_code_sha256(),
        # this kernel's own code + descriptor (PC-relative displacements masked): stays
        # valid while other kernels change
        "kernel_code_sha256": kernel_code_sha256(kernel_symbol(KERNEL)),
        "source": "rocprofv3 --kernel-trace --pmc <one counter group per pass>, tools/run_pmc.sh",
        "counters": counters,
        "kernel_ms_per_pass": kernel_ms,
        "fetch_bytes_corrected": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "notes": "FETCH_SIZE (KB) doubled per the gfx950 correction; WRITE_SIZE (KB) taken as is.",
    }
    c = counters
    if c.get("SQ_INSTS_VALU"):
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        out["valu_f64_fraction"] = f64 / c["SQ_INSTS_VALU"]
    if c.get("SQ_WAVE_CYCLES"):
        out["active_valu_over_wave_cycles"] = c.get("SQ_ACTIVE_INST_VALU", 0.0) / c["SQ_WAVE_CYCLES"]
        out["wait_inst_any_over_wave_cycles"] = c.get("SQ_WAIT_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        out["lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
