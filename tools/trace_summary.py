"""Per-kernel average durations (us) from a rocprofv3 --kernel-trace sqlite database."""
import collections
import sqlite3
import sys

for path in sys.argv[1:]:
    db = sqlite3.connect(path)
    rows = db.execute("select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join "
                      "rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    st = collections.defaultdict(list)
    for a, b, n in rows:
        st[n.split('(')[0]].append(b - a)
    print(path)
    for n, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:70]:70s} n={len(v):5d} avg={sum(v) / len(v) / 1000:9.2f} us")
