"""Per-launch summary of a rocprofv3 kernel trace (gpurun_out/<tag>/prof_*/run_kernel_trace.csv):
the flow kernel's launches in order, the mean over all of them and over the timed tail
(the clock ramps up over the first launches; bench.py's HIP-event timing covers the tail).

    python tools/trace_summary.py gpurun_out/r02m/prof_fwd/run_kernel_trace.csv lf_flow_kernel > out.json
"""
import csv
import json
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    tail = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ms = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if name in row["Kernel_Name"]:
                ms.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    out = {"kernel": name, "launches": len(ms), "mean_ms_all": sum(ms) / len(ms),
           f"mean_ms_last_{tail}": sum(ms[-tail:]) / len(ms[-tail:]), "min_ms": min(ms), "max_ms": max(ms),
           "per_launch_ms": [round(x, 4) for x in ms]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
