"""Per-step kernel timeline from a rocprofv3 --kernel-trace rocpd database: durations and
the idle gap before each dispatch (host-side stalls show up as gaps)."""
import sqlite3
import sys

db = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_project3d_fwd"
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if anchor in r[0]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
prev = None
busy = 0.0
for r in rows[i0:i1]:
    gap = (r[1] - prev) / 1000 if prev else 0.0
    busy += (r[2] - r[1]) / 1000
    print(f"{r[0][:52]:52s} dur={(r[2] - r[1]) / 1000:8.2f} gap_before={gap:7.2f}")
    prev = r[2]
span = (rows[i1][1] - rows[i0][1]) / 1000
print(f"step span {span:.1f} us, kernels {busy:.1f} us, idle {span - busy:.1f} us")
