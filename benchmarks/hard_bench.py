"""The hard (overlapping-blobs) regime of bench.py on its own: 2M x 256,
k = 1024, 1024 blobs in [-0.1, 0.1]^256 with spread 0.4 (mean delta-band ~3.8
members).  Prints bench.py's hard_* extras as one JSON line; meant to run
under rocprofv3 (scripts/prof_hard.sh) for the per-kernel table of the
regime."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000, help="bench --rows (the regime uses rows / 5)")
    ap.add_argument("--unpruned", action="store_true", help="also time the bounds-off engine")
    a = ap.parse_args()
    args = bench.parse(["--rows", str(a.rows)])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    extra = {}
    bench._hard_extra(extra, args, Comm(None), dev, unpruned=a.unpruned)
    print(json.dumps(extra), flush=True)


if __name__ == "__main__":
    main()
