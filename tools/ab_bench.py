"""Dev A/B of schedule knobs: runs bench.py once per environment setting (one process each, same box) and prints LM it/s,
ms per step and the factorization's HIP-event time. Settings are given as NAME=VALUE[,NAME=VALUE...] (or '-' for the
defaults); the first argument is the bench config.
    python tools/ab_bench.py C3 - G2OHIP_CHOL_PB=512 G2OHIP_SYRK_DMA=0 --steps 4
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv):
    cfg = argv[0]
    extra = []
    sets = []
    it = iter(argv[1:])
    for a in it:
        if a.startswith("--"):
            extra += [a, next(it)]
        else:
            sets.append(a)
    for s in sets or ["-"]:
        env = dict(os.environ)
        if s != "-":
            for kv in s.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        cmd = [sys.executable, os.path.join(HERE, "bench.py"), "--config", cfg, "--no-cpu-baseline", "--no-posegraph",
               "--no-c5"] + (extra or ["--steps", "6", "--warmup", "2"])
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            print(f"{s}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            return r.returncode
        d = json.loads(r.stdout.strip().splitlines()[-1])
        st = d.get("stages_ms_avg", {})
        print(f"{cfg} {s:60s} {d['value']:9.3f} LM it/s  {d['ms_per_step']:8.3f} ms/step  factor "
              f"{d['roofline']['avg_launch_ms']:8.3f} ms  schur_rows {st.get('schur_rows', 0):.3f}  "
              f"linearize {st.get('linearize', 0):.3f}  vreduce {st.get('vreduce', 0):.3f}  backsub {st.get('backsub', 0):.3f}  "
              f"trials {d['config']['levenberg_trials']}  ms/linear-solve {d.get('ms_per_linear_solve', 0):.3f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
