"""Print the end-to-end 2D -> 3D parity figures (tests/parity3d.py) of the HIP chain against the oracle
chain: config 2 (one frame, 8 views x 4 individuals) and a config-4 slice of --frames frames.
python tools/parity3d_probe.py [--frames 24] [--seeds 7,8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--seeds", default="7")
    a = ap.parse_args()
    import parity3d
    w = parity3d.make_weights()
    for seed in [int(s) for s in a.seeds.split(",")]:
        for nf in (1, a.frames):
            t = time.time()
            fig, _, _ = parity3d.run(n_frames=nf, seed=seed, weights=w)
            fig.update(n_frames=nf, seed=seed, seconds=round(time.time() - t, 1))
            print(json.dumps(fig), flush=True)


if __name__ == "__main__":
    main()
