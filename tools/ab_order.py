"""A/B of the profile-guided processing order: k_pulses<MU>/<MS> kernel time
(tools/time_mu.py) per corpus (bench, dense, zipf) under
  lpt    the shipped order: MU clock groups by descending MU_COST_KCYC cost, cut at 60 kcyc;
         MS protocols by descending MS_COST_KCYC
  clock  no cost model: MU groups in clock order, unsplit; MS in bank order
  size   the round-2 order: MU largest group first, unsplit; MS in bank order
Each (corpus, order) runs in its own process (the order is fixed when the bank is compiled),
``reps`` times, interleaved.  usage: python tools/ab_order.py [n] [reps]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ORDERS = {"lpt": {}, "clock": {"SDX_MU_ORDER": "clock", "SDX_MU_SPLIT": "0", "SDX_MS_ORDER": "bank"},
          "size": {"SDX_MU_ORDER": "size", "SDX_MU_SPLIT": "0", "SDX_MS_ORDER": "bank"}}


def main():
    n = sys.argv[1] if len(sys.argv) > 1 else "333333"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    for corpus in ("bench", "dense", "zipf"):
        for rep in range(1, reps + 1):
            for name, env in ORDERS.items():
                e = dict(os.environ, SDX_CORPUS=corpus, **env)
                r = subprocess.run([sys.executable, os.path.join(HERE, "time_mu.py"), n, "5"], env=e,
                                   capture_output=True, text=True, timeout=300)
                line = (r.stdout.strip().splitlines() or ["(no output) " + r.stderr[-300:]])[-1]
                print(f"{corpus:6s} {name:6s} rep{rep}: {line}", flush=True)
                if r.returncode:
                    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
