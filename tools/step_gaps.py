"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv):
durations and the idle gap before each dispatch (host-side stalls show up as gaps)."""
import csv
import sys

rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        for r in csv.DictReader(open(sys.argv[1]))]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_project3d_fwd"
rows.sort(key=lambda r: r[1])
idx = [i for i, r in enumerate(rows) if anchor in r[0]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
prev, busy = None, 0.0
for r in rows[i0:i1]:
    gap = (r[1] - prev) / 1000 if prev else 0.0
    busy += (r[2] - r[1]) / 1000
    print(f"{r[0][:50]:50s} dur={(r[2] - r[1]) / 1000:8.2f} gap={gap:7.2f}")
    prev = r[2]
span = (rows[i1][1] - rows[i0][1]) / 1000
print(f"step span {span:.1f} us, kernels {busy:.1f} us, idle {span - busy:.1f} us")
