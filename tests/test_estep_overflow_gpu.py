"""Dense rows of the certified E-step (csrc/estep_f32.hip): the 3-pass
kernel's overflow rows (a lane with a 3rd band member) get a second 3-pass
with three members per lane before the fp64 rows kernel.  Same delta-band
rule and Philox word, and every band decision of the 3-pass kernels is
certified (a value within the kernel's error bound of the band edge goes to
the fp64 re-check): the labels equal the fp64-only overflow path's bit for
bit, and the second pass does take most overflow rows."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.utils.datasets import make_blobs_device

pytestmark = pytest.mark.gpu


def _labels(monkeypatch, ovf2, X, C0):
    monkeypatch.setenv("SQ_OVF2", "1" if ovf2 else "0")
    eng = LloydEngine(X, C0.shape[0], delta=0.5, intermediate_error=True, seed=3)
    assert eng.fast and eng.certified
    eng.set_centers(C0)
    lab, mind, _ = eng.estep()
    torch.cuda.synchronize()
    return lab.clone().cpu(), mind.clone().cpu(), eng.buf.counts.clone().cpu()


def test_second_overflow_pass_matches_fp64_path(monkeypatch):
    n, d, k = 60000, 128, 1024
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=0.4, center_box=(-0.1, 0.1), seed=11,
                             device=torch.device("cuda"), dtype=torch.float32)
    rs = np.random.RandomState(11)
    C0 = X[torch.from_numpy(rs.choice(n, k, replace=False)).cuda()].clone()
    la, ma, ca = _labels(monkeypatch, True, X, C0)
    lb, mb, cb = _labels(monkeypatch, False, X, C0)
    assert int(ca[1]) > 0 and int(ca[0]) > 0          # dense rows, first-pass overflow rows
    assert int(ca[6]) < int(ca[0])                    # the second pass resolved some
    assert torch.equal(la, lb), int((la != lb).sum())
    assert torch.allclose(ma, mb, rtol=1e-6, atol=1e-5)
