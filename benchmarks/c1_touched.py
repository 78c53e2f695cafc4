"""How sparse could the C1 all-reduce bucket be?  Per headline iteration
(delta-means, 10M x 256, k = 1024, delta = 0.5) and per N = 8 shard (the
first 1.25M rows): rows whose label changed and the clusters they touch
(old or new label) - a compact (id, delta-sum, delta-count) bucket would
carry (d + 2) x 8 B per touched cluster instead of the dense k (d + 1) + 1
fp64 words."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def main():
    n, d, k, seed = 10_000_000, 256, 1024, 2024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=seed, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    for rows in (n, n // 8):
        eng = LloydEngine(X[:rows], k, delta=0.5, true_distance_estimate=False,
                          intermediate_error=True, true_tomography=False, seed=seed,
                          comm=Comm(None), gemm_precision="fp32")
        eng.set_centers(C0)
        prev = None
        out = []
        for s in range(14):
            lab = eng.step()[0].clone()
            if prev is not None and s >= 4:
                ch = lab != prev
                nch = int(ch.sum())
                touched = int(torch.unique(torch.cat([lab[ch], prev[ch]]).long()).numel())
                out.append({"step": s, "changed_rows": nch, "touched_clusters": touched,
                            "compact_bytes_frac": touched * (d + 2) / (k * (d + 1) + 1)})
            prev = lab
        print(json.dumps({"rows": rows, "steps": out}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
