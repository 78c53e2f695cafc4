"""Batched k-means++ restarts (ops.kmeans.KmppBatch) vs one sequential
restart on the bench data (10M x 256 blobs, k = 1024, t = 2 + ln k):
seconds per restart."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data  # noqa: E402
from sq_learn_amd.models.cluster import _init as I  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
RS = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 4, 10]
dev = torch.device("cuda")
X, _ = make_blobs_device(n, 256, centers=1024, cluster_std=1.0, seed=2024, device=dev,
                         dtype=torch.float32)
X -= X.mean(0, keepdim=True)
data = Data(X, n, 0, Comm(None), "sharded")
I.kmeans_plusplus(data, k, np.random.RandomState(0))      # warm
torch.cuda.synchronize()
t0 = time.perf_counter()
I.kmeans_plusplus(data, k, np.random.RandomState(1))
torch.cuda.synchronize()
out = {"sequential_s_per_restart": time.perf_counter() - t0}
for R in RS:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    I.kmeans_plusplus_restarts(data, k, np.random.RandomState(1), R)
    torch.cuda.synchronize()
    out[f"batched{R}_s_per_restart"] = (time.perf_counter() - t0) / R
print(json.dumps(out), flush=True)
