"""Same-box A/B of the 3D projection's optional isect_count output (round 6): runs bench.py with
render._counts3d on (the counts written, as before) and off (NULL, the product path), one library.
Usage (on the GPU box): python3 tools/ab_counts3d.py CONFIG REPS [bench args...]"""
import json
import os
import runpy
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode: str, argv):
    sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
    sys.path.insert(0, ROOT)
    import gsr.render as R
    R._counts3d = mode == "on"
    sys.argv = ["bench.py"] + argv
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3:])
        return
    cfg, reps, extra = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    steps = ["--steps", "20", "--warmup", "3"] if cfg == "5" else ["--steps", "40", "--warmup", "5"]
    for r in range(reps):
        for mode in ("on", "off"):
            argv = ["--config", cfg, "--cpu-baseline", "0", "--psnr", "0"] + steps + extra
            out = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", mode] + argv,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            k = d.get("kernels_ms", {})
            print(f"c{cfg} counts {mode} #{r + 1}", round(d["value"], 1), round(d["ms_per_step"], 4), "ms",
                  {x: k[x] for x in k if "project" in x}, flush=True)


if __name__ == "__main__":
    main()
