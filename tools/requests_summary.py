"""Summary of tools/gpu_requests.sh: per kernel, the L2 -> HBM write requests (all, 64-B,
atomics) and read requests of one frame, beside the integrate -> shade hand-off bytes of
the same frame (tools/handoff_bytes.py).  A write request moves 64 B (the _64B ones) or
up to 128 B (the rest), a read request 64 B on gfx950 (FETCH_SIZE = RDREQ x 64 B;
/opt/skills/guides/MI355X_MICROARCH.md).

python3 tools/requests_summary.py gpurun_out/<tag> c2 [c3 ...] > profiles/<tag>/requests.json"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def counters(path):
    out = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        out[name][row["Counter_Name"]] += float(row["Counter_Value"])
    return out


def summary(d, w):
    wr = counters(d / f"{w}_wr" / "run_counter_collection.csv")
    rd = counters(d / f"{w}_rd" / "run_counter_collection.csv")
    hand = json.loads((d / f"{w}_handoff.json").read_text().strip().splitlines()[-1])
    kernels = {}
    for k in sorted(set(wr) | set(rd)):
        if k.startswith("__amd"):
            continue
        c = dict(wr.get(k, {}))
        c.update(rd.get(k, {}))
        n_wr, n64, n_at = c.get("TCC_EA0_WRREQ_sum", 0.0), c.get("TCC_EA0_WRREQ_64B_sum", 0.0), c.get(
            "TCC_EA0_ATOMIC_sum", 0.0)
        kernels[k] = {"wrreq": n_wr, "wrreq_64B": n64, "atomics": n_at, "rdreq": c.get("TCC_EA0_RDREQ_sum", 0.0),
                      # 64-B requests move 64 B, the others up to 128 B
                      "write_bytes_max": 64 * n64 + 128 * (n_wr - n64),
                      "read_bytes": 64 * c.get("TCC_EA0_RDREQ_sum", 0.0)}
    return {"workload": w, "handoff": hand, "kernels": kernels}


if __name__ == "__main__":
    d = Path(sys.argv[1])
    print(json.dumps({"source": str(d), "frames": [summary(d, w) for w in sys.argv[2:]]}, indent=1))
