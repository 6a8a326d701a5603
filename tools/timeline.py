"""Dev helper: the last N kernels of a rocprofv3 kernel trace as a per-scan timeline (µs from the
first shown), with queue ids — shows inter-kernel gaps. Usage: python3 tools/timeline.py <kernel_trace.csv> [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sel = rows[-(int(sys.argv[2]) if len(sys.argv) > 2 else 12):]
t0 = int(sel[0]["Start_Timestamp"])
prev = None
for r in sel:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    gap = "" if prev is None else f"gap {s - prev:6.1f}"
    print(f"{r['Kernel_Name'][:40]:40s} q={r['Queue_Id']:>2s} {s:8.1f} {e:8.1f} dur {e - s:7.1f} {gap}")
    if r["Queue_Id"] == sel[-1]["Queue_Id"] or prev is None:
        prev = e
