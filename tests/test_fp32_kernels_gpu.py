"""fp32-mode kernels (the reference model run without autocast) vs fp64 references of the same op.

Every kernel here is reached through the same _lib wrappers as the bf16 path: fp32 tensors select
the *_f32 entry points of include/gpt2mi.h. Tolerances are at fp32 accumulation-order resolution."""
import pytest
import torch

from oracle import model_ref

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpt_2_distributed_amd import _lib
    _lib.load()


def L():
    from gpt_2_distributed_amd import _lib
    return _lib


def rel_err(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _ref(layout, A, B):
    A, B = A.double(), B.double()
    return A @ B.t() if layout == 0 else (A @ B if layout == 1 else A.t() @ B)


@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(128, 128, 16), (200, 384, 768), (512, 260, 48), (64, 2304, 128)])
def test_gemm_f32_layouts(layout, M, N, K):
    g = torch.Generator().manual_seed(M + 3 * N + K + layout)
    if layout == 0:
        A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    elif layout == 1:
        A, B = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
    else:
        A, B = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(dev)
    L().gemm(layout, L().EPI_F32, M, N, K, A.to(dev), A.shape[1], B.to(dev), B.shape[1], C, N, alpha=0.5,
             accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(C.cpu(), C0.double() + 0.5 * _ref(layout, A, B)) < 2e-6


def test_gemm_f32_epilogues():
    M, N, K = 192, 512, 256
    g = torch.Generator().manual_seed(3)
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    bias, resid = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    acc = _ref(0, A, W)
    Ad, Wd = A.to(dev), W.to(dev)
    C = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, K, Ad, K, Wd, K, C, N, bias=bias.to(dev))  # "BF16" = activation dtype
    assert rel_err(C.cpu(), acc + bias.double()) < 2e-6
    Cr = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_RESID, M, N, K, Ad, K, Wd, K, Cr, N, bias=bias.to(dev), resid=resid.to(dev))
    assert rel_err(Cr.cpu(), resid.double() + acc + bias.double()) < 2e-6
    Cg, G = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_GELU, M, N, K, Ad, K, Wd, K, Cg, N, bias=bias.to(dev), aux=G, ldaux=N)
    u = (acc + bias.double()).requires_grad_(True)
    assert rel_err(Cg.cpu(), model_ref.gelu_tanh(u.detach())) < 1e-5
    # GELU backward through the fc2 dgrad: dU = (dY @ W2) * gelu'(u), gelu'(u) emitted by the forward
    dY, W2 = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g) * 0.05
    dU = torch.empty(M, N, device=dev)
    L().gemm(1, L().EPI_GELU_BWD, M, N, K, dY.to(dev), K, W2.to(dev), N, dU, N, aux=G, ldaux=N)
    model_ref.gelu_tanh(u).backward(_ref(1, dY, W2))
    assert rel_err(dU.cpu(), u.grad) < 1e-5


def test_gemm_f32_dropout_mask_matches_bf16_kernel():
    """Both precisions drop the same elements (same (seed, element) hash)."""
    M, N, K, p = 256, 256, 64, 0.25
    A, W, R = torch.randn(M, K), torch.randn(N, K), torch.zeros(M, N)
    c32 = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_RESID, M, N, K, A.to(dev), K, W.to(dev), K, c32, N, resid=R.to(dev), p_drop=p, seed=77)
    c16 = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_RESID, M, N, K, A.bfloat16().to(dev), K, W.bfloat16().to(dev), K, c16, N, resid=R.to(dev),
             p_drop=p, seed=77)
    assert torch.equal(c32 == 0, c16 == 0)
    frac = (c32 == 0).float().mean().item()
    assert abs(frac - p) < 0.02


@pytest.mark.parametrize("B,T,H", [(1, 64, 1), (2, 256, 3), (1, 1024, 2), (2, 128, 4)])
def test_attention_f32_fwd_bwd(B, T, H):
    D, C = 64, 64 * H
    g = torch.Generator().manual_seed(B * T + H)
    qkv = torch.randn(B * T, 3 * C, generator=g)
    q, k, v = [t.double().clone().requires_grad_(True) for t in qkv.view(B, T, 3, H, D).transpose(1, 3).unbind(2)]
    y = model_ref.causal_attention(q, k, v, "fp32")
    dy = torch.randn(B, H, T, D, generator=g)
    y.backward(dy.double())
    qd = qkv.to(dev)
    out = torch.empty(B * T, C, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    L().attn_fwd(qd, out, lse, B, T, H, D)
    torch.cuda.synchronize()
    assert rel_err(out.cpu(), y.detach().transpose(1, 2).reshape(B * T, C)) < 2e-6
    dout = dy.transpose(1, 2).reshape(B * T, C).contiguous().to(dev)
    dqkv = torch.empty(B * T, 3 * C, device=dev)
    delta = torch.empty(B * H, T, device=dev)
    L().attn_bwd(qd, out, dout, lse, delta, dqkv, B, T, H, D)
    torch.cuda.synchronize()
    dq, dk, dv = dqkv.cpu().view(B, T, 3, H, D).transpose(1, 3).unbind(2)
    assert rel_err(dq, q.grad) < 1e-5
    assert rel_err(dk, k.grad) < 1e-5
    assert rel_err(dv, v.grad) < 1e-5


def test_attention_f32_dropout_same_mask_as_bf16():
    """The expected dropped fraction is p and dV of a one-hot dO shows the same kept set for both
    precisions (same pair hash)."""
    B, T, H, D, p = 1, 128, 1, 64, 0.2
    g = torch.Generator().manual_seed(2)
    qkv = torch.randn(B * T, 3 * 64, generator=g) * 0.1
    outs = {}
    for name, x in (("f32", qkv), ("bf16", qkv.bfloat16())):
        xd = x.to(dev)
        o = torch.empty(B * T, 64, dtype=x.dtype, device=dev)
        lse = torch.empty(B * H, T, device=dev)
        L().attn_fwd(xd, o, lse, B, T, H, D, p, 31)
        # dV[key] = sum_q P_drop[q,key] dO[q]: with dO = ones on column 0 only the kept pattern matters
        dout = torch.zeros(B * T, 64, dtype=x.dtype, device=dev)
        dout[T - 1, 0] = 1.0  # last query sees every key
        dq = torch.empty(B * T, 3 * 64, dtype=x.dtype, device=dev)
        delta = torch.empty(B * H, T, device=dev)
        L().attn_bwd(xd, o, dout, lse, delta, dq, B, T, H, D, p, 31)
        outs[name] = dq[:, 2 * 64].float().cpu()
    assert torch.equal(outs["f32"] == 0, outs["bf16"] == 0)
    assert 0.05 < (outs["f32"] == 0).float().mean().item() < 0.4


def test_layernorm_bwd_and_colsum_f32():
    M, C = 256, 768
    g = torch.Generator().manual_seed(5)
    x, w, b = torch.randn(M, C, generator=g), torch.randn(C, generator=g) * 0.1 + 1, torch.randn(C, generator=g)
    dy, dres0 = torch.randn(M, C, generator=g), torch.randn(M, C, generator=g)
    xr, wr, br = (t.double().clone().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.layer_norm(xr, (C,), wr, br, 1e-5).backward(dy.double())
    xd, wd, bd = x.to(dev), w.to(dev), b.to(dev)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    y = torch.empty(M, C, device=dev)
    L().layernorm_fwd(xd, wd, bd, None, y, mean, rstd, M, C, 1e-5)
    dres = dres0.to(dev)
    dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    out, dbo = torch.empty(M, C, device=dev), torch.zeros(C, device=dev)
    L().layernorm_bwd(xd, wd, mean, rstd, dy.to(dev), dres, dw, db, out, dbo, M, C)
    torch.cuda.synchronize()
    assert rel_err(dres.cpu(), dres0.double() + xr.grad) < 1e-5
    assert rel_err(dw.cpu(), wr.grad) < 1e-5 and rel_err(db.cpu(), br.grad) < 1e-5
    assert torch.equal(out, dres)  # p = 0: the branch grad is the residual grad, in fp32
    assert rel_err(dbo.cpu(), dres.cpu().double().sum(0)) < 1e-5
    cs = torch.ones(C, device=dev)
    L().colsum_bf16(dres, cs, M, C, C)
    assert rel_err(cs.cpu(), 1 + dres.cpu().double().sum(0)) < 1e-6


def test_xent_f32():
    M, V, ld = 96, 50257, 50432
    g = torch.Generator().manual_seed(8)
    logits = torch.randn(M, ld, generator=g) * 3
    labels = torch.randint(0, V, (M,), generator=g)
    lg = logits[:, :V].double().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lg, labels)
    ref.backward()
    rows, lse = torch.empty(M, device=dev), torch.empty(M, device=dev)
    dl = torch.empty(M, ld, device=dev)
    loss, inv = torch.empty(1, device=dev), torch.empty(1, device=dev)
    L().xent_fwd(logits.to(dev), ld, labels.to(dev), rows, lse, dl, ld, M, V, loss, inv)
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 2e-6 * ref.item()
    assert rel_err(dl.cpu()[:, :V] * inv.item(), lg.grad) < 1e-5
    assert torch.all(dl[:, V:] == 0)
