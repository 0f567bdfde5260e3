"""A/B timing of libccmpc.so builds on the bandwidth/latency configs (GPU box, repo root):

    python tools/ab_configs.py main build_d3 build_d4      (names: csrc/<name>/libccmpc.so;
                                                            "main" = the in-tree library)

Each variant runs in its own child process (the library is loaded once per process) and
prints one line per config: the one-launch cycle and the moments-only launch, warm (back to
back on one store) and cold (rotating over distinct stores, bench.cold_time).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [("C2", 4, 5000, 8, 1), ("C3-1e3", 1, 1000, 8, 1), ("C3-2e4", 1, 20000, 8, 1),
           ("C3-1e5", 1, 100000, 8, 1), ("C4/8", 4, 20000, 12, 8), ("C4/1", 4, 20000, 12, 64),
           ("C5", 8, 50000, 40, 1), ("C4/8-f32", 4, 20000, 12, 8), ("C4/1-f32", 4, 20000, 12, 64)]


def child(only):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
    import torch
    import bench
    dev = torch.device("cuda", 0)
    for name, O, N, T, scenes in CONFIGS:
        if only and name not in only:
            continue
        row = bench.time_config(dev, 20251015, name, O, N, T, scenes,
                                cold=N * O * scenes * T * 16 >= (8 << 20),
                                f32=name.endswith("-f32"))
        print(json.dumps(row), flush=True)
        torch.cuda.empty_cache()


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2:])
        return
    only = os.environ.get("ONLY", "").split(",") if os.environ.get("ONLY") else []
    for v in sys.argv[1:]:
        env = dict(os.environ)
        if v != "main":
            env["CCMPC_LIB"] = os.path.join(ROOT, "cc-mpc_amd", "csrc", v, "libccmpc.so")
        print(f"== {v}", flush=True)
        r = subprocess.run([sys.executable, __file__, "--child"] + only, env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300)
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                d = json.loads(line)
                print(f"  {d['config']:8s} cycle {d['kernel_us']:8.2f}  mom {d['moments_only_us']:8.2f}"
                      f"  frac {d['frac']:.3f}  cold {d.get('cold_kernel_us', float('nan')):8.2f}"
                      f"  cold_frac {d.get('cold_frac', float('nan')):.3f}", flush=True)
        if r.returncode != 0:
            print(r.stdout[-3000:])
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
