"""RotatE training gradients on the HIP path (rnnl_rotate_backward through
embedding._RotatEScore) against torch autograd of the reference's
arithmetic (RotatE.forward_torch, embedding.py:45-70): eemb and remb
gradients for a random upstream gradient, including a row whose target
entity equals h under a zero-phase relation (|h o r - t| = 0 in every dim:
torch.norm's zero-gradient convention)."""
import numpy as np
import pytest
import torch

from conftest import Fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["umls_emb_pna_rotate", "fb_lstm_sum_rotate"])
def test_rotate_backward_matches_torch(case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnlogic_amd.embedding import RotatE
    fx = Fixture(case)
    dev = torch.device("cuda:0")
    rot = RotatE(fx.rotate_path()).to(dev)
    E, R2 = rot.num_entities, rot.remb.size(0)
    gen = torch.Generator().manual_seed(0)
    B = 32
    h = torch.randint(0, E, (B,), generator=gen).to(dev)
    r = torch.randint(0, R2, (B,), generator=gen).to(dev)
    with torch.no_grad():
        rot.remb[int(r[0])].zero_()  # row 0: h o r == h, so the target h has distance 0
    g = torch.randn(B, E, generator=gen).to(dev)
    grads = []
    for fn in (rot.forward_torch, rot.forward_grad):
        rot.zero_grad()
        s = fn(h, r)
        (s * g).sum().backward()
        grads.append((s.detach().clone(), rot.eemb.grad.clone(), rot.remb.grad.clone()))
    # float64 autograd of the same arithmetic: the yardstick for both fp32 paths
    rot64 = RotatE(fx.rotate_path()).to(dev).double()
    with torch.no_grad():
        rot64.remb[int(r[0])].zero_()
    (rot64.forward_torch(h, r) * g.double()).sum().backward()
    (s0, ge0, gr0), (s1, ge1, gr1) = grads
    assert float((s0 - s1).abs().max()) <= 1e-4
    for name, a, b, w in (("eemb", ge0, ge1, rot64.eemb.grad), ("remb", gr0, gr1, rot64.remb.grad)):
        a, b, w = a.cpu().numpy(), b.cpu().numpy(), w.cpu().numpy()
        assert np.isfinite(b).all(), name
        err = float(np.abs(a - b).max())
        scale = float(np.abs(a).max())
        e_hip, e_torch = float(np.abs(b - w).max()), float(np.abs(a - w).max())
        print("%s %s grad: max |hip - torch| %.3g, |hip - f64| %.3g, |torch - f64| %.3g (max |grad| %.3g)"
              % (case, name, err, e_hip, e_torch, scale))
        # within the fp32 torch path's own distance from float64 (x 2), or the
        # tolerance of the element-wise comparison with it
        if e_hip > 2 * e_torch:
            np.testing.assert_allclose(b, a, atol=1e-5 * scale + 1e-6, rtol=1e-4, err_msg=name)
