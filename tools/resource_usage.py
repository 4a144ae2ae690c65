"""Parse hipcc -Rpass-analysis=kernel-resource-usage remarks from stdin: one line per kernel."""
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "?"
cur = {}
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    key, val = m.groups()
    key = key.split()[0]
    if key == "Function":
        cur = {"name": val}
        continue
    cur[key] = val
    if key == "LDS":
        print(f"{src:16s} {cur['name'][:72]:72s} vgpr {cur.get('VGPRs')} scratch {cur.get('ScratchSize')} "
              f"occ {cur.get('Occupancy')} lds {val}")
