"""Per-kernel parity on the MI355X: each HIP kernel (through the C ABI) vs the oracle / a plain
PyTorch fp32 reference of the same op on the same seeded inputs. Tolerances are written per test:
bf16 outputs are compared at bf16 resolution, fp32 outputs at accumulation-order resolution."""
import math

import pytest
import torch

from oracle import model_ref, train_ref

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpt_2_distributed_amd import _lib
    _lib.load()
    return _lib


def L():
    from gpt_2_distributed_amd import _lib
    return _lib


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("M,C", [(256, 768), (128, 128), (64, 1600), (200, 1024)])
def test_layernorm_fwd_bwd(M, C):
    g = torch.Generator(device="cpu").manual_seed(M + C)
    x = torch.randn(M, C, generator=g) * 2 + 0.5
    w = torch.randn(C, generator=g) * 0.1 + 1
    b = torch.randn(C, generator=g) * 0.1
    dy = bf(torch.randn(M, C, generator=g))
    dres0 = torch.randn(M, C, generator=g)
    # oracle
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = model_ref.layer_norm(xr, wr, br, 1e-5)
    y.backward(dy.float())
    # HIP
    xd, wd, bd = x.to(dev), w.to(dev), b.to(dev)
    yb = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    yf = torch.empty(M, C, device=dev)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    L().layernorm_fwd(xd, wd, bd, yb, yf, mean, rstd, M, C, 1e-5)
    torch.cuda.synchronize()
    assert rel_err(yf.cpu(), y.detach()) < 1e-6
    assert (yb.cpu().float() - bf(y.detach()).float()).abs().max() <= 2 ** -7 * y.detach().abs().max()
    dres = dres0.to(dev).clone()
    dw = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    outb = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    dbo = torch.zeros(C, device=dev)
    L().layernorm_bwd(xd, wd, mean, rstd, dy.to(dev), dres, dw, db, outb, dbo, M, C)
    torch.cuda.synchronize()
    ref_dres = dres0 + xr.grad
    assert rel_err(dres.cpu(), ref_dres) < 1e-5
    assert rel_err(dw.cpu(), wr.grad) < 1e-5
    assert rel_err(db.cpu(), br.grad) < 1e-5
    assert rel_err(outb.cpu().float(), ref_dres) < 5e-3
    assert rel_err(dbo.cpu(), outb.cpu().float().sum(0)) < 1e-5


def test_embed_fwd_bwd():
    B, T, C, V = 4, 64, 768, 1000
    g = torch.Generator().manual_seed(1)
    idx = torch.randint(0, V, (B, T), generator=g)
    wte = torch.randn(V, C, generator=g)
    wpe = torch.randn(T, C, generator=g)
    x = torch.empty(B * T, C, device=dev)
    L().embed_fwd(idx.to(dev), wte.to(dev), wpe.to(dev), x, B, T, C)
    ref = model_ref.embed(wte, wpe, idx).reshape(B * T, C)
    assert torch.equal(x.cpu(), ref)
    dres = torch.randn(B * T, C, generator=g)
    dwte = torch.zeros(V, C, device=dev)
    dwpe = torch.zeros(T, C, device=dev)
    L().embed_bwd(idx.to(dev), dres.to(dev), dwte, dwpe, B, T, C)
    rw = torch.zeros(V, C).index_add_(0, idx.reshape(-1), dres)
    rp = dres.reshape(B, T, C).sum(0)
    assert rel_err(dwte.cpu(), rw) < 1e-6
    assert rel_err(dwpe.cpu(), rp) < 1e-6


def test_embed_dropout_mask_consistent():
    B, T, C, V, p = 2, 64, 256, 100, 0.1
    idx = torch.randint(0, V, (B, T))
    wte = torch.randn(V, C, device=dev).abs() + 0.1
    wpe = torch.randn(T, C, device=dev).abs() + 0.1
    x = torch.empty(B * T, C, device=dev)
    L().embed_fwd(idx.to(dev), wte, wpe, x, B, T, C, p, 1234)
    kept = x != 0
    frac = 1 - kept.float().mean().item()
    assert abs(frac - p) < 0.01
    base = (wte[idx.to(dev)] + wpe.unsqueeze(0)).reshape(B * T, C)
    torch.testing.assert_close(x[kept], base[kept] / (1 - p))
    # backward regenerates the same mask: grads of dropped elements do not reach the tables
    dres = torch.ones(B * T, C, device=dev)
    dwpe = torch.zeros(T, C, device=dev)
    dwte = torch.zeros(V, C, device=dev)
    L().embed_bwd(idx.to(dev), dres, dwte, dwpe, B, T, C, p, 1234)
    exp = (kept.float() / (1 - p)).reshape(B, T, C).sum(0)
    torch.testing.assert_close(dwpe, exp)


def _gemm_ref(layout, A, B):
    Af, Bf = A.float(), B.float()
    if layout == 0:
        return Af @ Bf.t()
    if layout == 1:
        return Af @ Bf
    return Af.t() @ Bf


@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 768), (512, 256, 192),
                                   # half-width last tiles (C = 1600 of GPT-2 1.5B: N = 1600, 4800)
                                   (192, 192, 128), (320, 576, 192)])
def test_gemm_layouts_f32(layout, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K + layout)
    if layout == 0:
        A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    elif layout == 1:
        A, B = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
    else:
        A, B = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
    A, B = bf(A), bf(B)
    ref = _gemm_ref(layout, A, B)
    C = torch.zeros(M, N, device=dev)
    Ad, Bd = A.to(dev), B.to(dev)
    lda, ldb = A.shape[1], B.shape[1]
    epi = L().EPI_F32 if layout != 2 else L().EPI_ATOMIC
    L().gemm(layout, epi, M, N, K, Ad, lda, Bd, ldb, C, N, alpha=0.5)
    torch.cuda.synchronize()
    assert rel_err(C.cpu(), 0.5 * ref) < 1e-5


def test_gemm_wgrad_splitk_accumulate():
    M, N, K = 256, 384, 1024
    A, B = bf(torch.randn(K, M)), bf(torch.randn(K, N))
    C0 = torch.randn(M, N)
    C = C0.to(dev)
    L().gemm(2, L().EPI_ATOMIC, M, N, K, A.to(dev), M, B.to(dev), N, C, N, splits=4)
    assert rel_err(C.cpu(), C0 + A.float().t() @ B.float()) < 1e-5


def test_gemm_epilogues_forward():
    M, N, K = 256, 512, 256
    g = torch.Generator().manual_seed(3)
    A, W = bf(torch.randn(M, K, generator=g)), bf(torch.randn(N, K, generator=g) * 0.05)
    bias = torch.randn(N, generator=g)
    resid = torch.randn(M, N, generator=g)
    acc = A.float() @ W.float().t()
    Ad, Wd = A.to(dev), W.to(dev)
    # BF16 + bias
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, K, Ad, K, Wd, K, C, N, bias=bias.to(dev))
    assert rel_err(C.cpu().float(), acc + bias) < 4e-3
    # RESID
    Cr = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_RESID, M, N, K, Ad, K, Wd, K, Cr, N, bias=bias.to(dev), resid=resid.to(dev))
    assert rel_err(Cr.cpu(), resid + acc + bias) < 1e-5
    # GELU: C = gelu(u), aux = gelu'(u) (no dropout: keep = 1)
    Cg = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    G = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_GELU, M, N, K, Ad, K, Wd, K, Cg, N, bias=bias.to(dev), aux=G, ldaux=N)
    u = (acc + bias).requires_grad_(True)
    model_ref.gelu_tanh(u).sum().backward()
    assert rel_err(G.cpu().float(), u.grad) < 4e-3
    assert rel_err(Cg.cpu().float(), model_ref.gelu_tanh(u.detach())) < 4e-3


def test_gemm_gelu_bwd_dgrad():
    """fc1 forward (EPI_GELU, with dropout) then fc2 dgrad (EPI_GELU_BWD) reproduce autograd of
    drop(gelu(u)): dU = (dY @ W2) * keep/(1-p) * gelu'(u), with the mask regenerated nowhere."""
    M, N, K = 256, 256, 384  # u[M,N] = X[M,K'] W1^T ; dH[M,N] = dY[M,K] @ W2[K,N]
    g = torch.Generator().manual_seed(4)
    X, W1 = bf(torch.randn(M, 128, generator=g)), bf(torch.randn(N, 128, generator=g) * 0.1)
    dY, W2 = bf(torch.randn(M, K, generator=g)), bf(torch.randn(K, N, generator=g) * 0.05)
    p = 0.25
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    G = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_GELU, M, N, 128, X.to(dev), 128, W1.to(dev), 128, H, N, aux=G, ldaux=N, p_drop=p, seed=9)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(1, L().EPI_GELU_BWD, M, N, K, dY.to(dev), K, W2.to(dev), N, C, N, aux=G, ldaux=N)
    keep = (H.cpu().float() != 0).float()  # gelu(u) != 0 almost surely: the kept set
    assert abs(1 - keep.mean().item() - p) < 0.03
    u = (X.float() @ W1.float().t()).requires_grad_(True)
    (model_ref.gelu_tanh(u) * keep / (1 - p)).backward(dY.float() @ W2.float())
    assert rel_err(C.cpu().float(), u.grad) < 1e-2


def test_gemm_rejects_bad_shapes():
    from gpt_2_distributed_amd._lib import KernelError
    A = torch.zeros(128, 128, dtype=torch.bfloat16, device=dev)
    with pytest.raises(KernelError, match="multiples of 64"):
        L().gemm(0, 0, 128, 100, 64, A, 128, A, 128, A, 128)
    with pytest.raises(KernelError, match="of 64"):
        L().gemm(0, 0, 100, 128, 64, A, 128, A, 128, A, 128)


def test_gemm_half_width_n_tile_epilogues():
    """N % 128 == 64 (GPT-2 1.5B widths; the 256x256 kernel's partial column tile, 3 K-tiles: its odd-count zero
    tile): bias / GELU+dropout / residual epilogues write exactly the N valid columns (the padding columns of a
    wider C stay untouched)."""
    M, N, K = 256, 320, 192
    g = torch.Generator().manual_seed(21)
    A, W = bf(torch.randn(M, K, generator=g)), bf(torch.randn(N, K, generator=g) * 0.1)
    bias, resid = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    acc = A.float() @ W.float().t() + bias
    Ad, Wd = A.to(dev), W.to(dev)
    ld = N + 64
    C = torch.full((M, ld), 3.0, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, K, Ad, K, Wd, K, C, ld, bias=bias.to(dev))
    assert rel_err(C[:, :N].cpu().float(), acc) < 4e-3
    assert torch.all(C[:, N:] == 3.0)
    Cr = torch.full((M, ld), 5.0, device=dev)
    Rd = torch.zeros(M, ld, device=dev)
    Rd[:, :N] = resid.to(dev)
    L().gemm(0, L().EPI_RESID, M, N, K, Ad, K, Wd, K, Cr, ld, bias=bias.to(dev), resid=Rd)
    assert rel_err(Cr[:, :N].cpu(), resid + acc) < 1e-5
    assert torch.all(Cr[:, N:] == 5.0)
    H = torch.full((M, ld), 3.0, dtype=torch.bfloat16, device=dev)
    G = torch.full((M, ld), 3.0, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_GELU, M, N, K, Ad, K, Wd, K, H, ld, bias=bias.to(dev), aux=G, ldaux=ld)
    assert rel_err(H[:, :N].cpu().float(), model_ref.gelu_tanh(acc)) < 4e-3
    assert torch.all(H[:, N:] == 3.0) and torch.all(G[:, N:] == 3.0)


def test_gemm_partial_m_tile():
    M, N, K = 192, 256, 128
    A, W = bf(torch.randn(M, K)), bf(torch.randn(N, K))
    C = torch.full((M + 64, N), 7.0, device=dev)
    L().gemm(0, L().EPI_F32, M, N, K, A.to(dev), K, W.to(dev), K, C, N)
    assert rel_err(C[:M].cpu(), A.float() @ W.float().t()) < 1e-5
    assert torch.all(C[M:] == 7.0)


def _attn_inputs(B, T, H, seed):
    D = 64
    C = H * D
    g = torch.Generator().manual_seed(seed)
    qkv = bf(torch.randn(B * T, 3 * C, generator=g))
    return qkv, C


def _attn_ref(qkv, B, T, H):
    D = 64
    C = H * D
    q, k, v = qkv.float().view(B, T, 3, H, D).transpose(1, 3).unbind(2)
    return q, k, v


# B*H % 8 == 0: every head stays on one XCD under the heaviest-first block map; the others spread over XCDs
@pytest.mark.parametrize("B,T,H", [(1, 64, 1), (2, 128, 2), (1, 1024, 2), (2, 256, 4), (4, 512, 6)])
def test_attention_fwd_bwd(B, T, H):
    D = 64
    qkv, C = _attn_inputs(B, T, H, B * T + H)
    q, k, v = [t.clone().requires_grad_(True) for t in _attn_ref(qkv, B, T, H)]
    y = model_ref.causal_attention(q, k, v, "fp32")  # [B,H,T,D]
    dy = bf(torch.randn(B, H, T, D))
    y.backward(dy.float())
    yref = y.detach().transpose(1, 2).reshape(B * T, C)
    out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    qd = qkv.to(dev)
    L().attn_fwd(qd, out, lse, B, T, H, D)
    torch.cuda.synchronize()
    assert rel_err(out.cpu().float(), yref) < 6e-3
    s = (q @ k.transpose(-2, -1)) / 8.0
    s = s.masked_fill(~torch.tril(torch.ones(T, T, dtype=torch.bool)), float("-inf"))
    # the kernel's normaliser is the sum of the bf16-rounded probabilities its PV product uses (row
    # sums by MFMA): |d lse| ~ 2^-9 / sqrt(3 * keys) relative, not fp32-exact
    assert rel_err(lse.cpu().view(B, H, T), torch.logsumexp(s.detach(), -1)) < 3e-4
    dout = dy.transpose(1, 2).reshape(B * T, C).contiguous().to(dev)
    dqkv = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * H, T, device=dev)
    L().attn_bwd(qd, out, dout, lse, delta, dqkv, B, T, H, D)
    torch.cuda.synchronize()
    dq, dk, dv = dqkv.cpu().float().view(B, T, 3, H, D).transpose(1, 3).unbind(2)
    assert rel_err(dq, q.grad) < 1e-2
    assert rel_err(dk, k.grad) < 1e-2
    assert rel_err(dv, v.grad) < 1e-2


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_bwd_fused_bias_grad_partials(p):
    """The backward's 32-token partial column sums of the stored dqkv (the qkv bias gradient, summed by
    colsum) equal the column sums of dqkv itself, and requesting them leaves dqkv unchanged."""
    B, T, H, D = 2, 256, 4, 64
    qkv, C = _attn_inputs(B, T, H, 77)
    qd = qkv.to(dev)
    out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    L().attn_fwd(qd, out, lse, B, T, H, D, p, 5)
    dout = bf(torch.randn(B * T, C, generator=torch.Generator().manual_seed(1))).to(dev)
    delta = torch.empty(B * H, T, device=dev)
    d1 = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
    d2 = torch.empty_like(d1)
    cs = torch.empty(B * T // 32, 3 * C, device=dev)
    L().attn_bwd(qd, out, dout, lse, delta, d1, B, T, H, D, p, 5)
    L().attn_bwd(qd, out, dout, lse, delta, d2, B, T, H, D, p, 5, colsum=cs)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)
    ref = d1.float().view(B * T // 32, 32, 3 * C).sum(1)
    assert rel_err(cs.cpu(), ref.cpu()) < 1e-5
    bias_grad = torch.zeros(3 * C, device=dev)
    L().colsum_bf16(cs, bias_grad, B * T // 32, 3 * C, 3 * C)
    assert rel_err(bias_grad.cpu(), d1.float().sum(0).cpu()) < 1e-5


def test_attention_backward_deterministic():
    """Repeated backwards of one forward at a full-size head count (B=8, T=1024, H=12, dropout 0.1) store the same
    bits: the software-pipelined dQ / dK-dV tiles once read MFMA results too early through an inline-asm select (a
    hazard the compiler does not pad for asm operands), which showed as run-to-run dK differences at p > 0 only."""
    B, T, H, D, p = 8, 1024, 12, 64, 0.1
    qkv, C = _attn_inputs(B, T, H, 4242)
    qd = qkv.to(dev)
    out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    L().attn_fwd(qd, out, lse, B, T, H, D, p, 11)
    dout = bf(torch.randn(B * T, C, generator=torch.Generator().manual_seed(2)) * 0.1).to(dev)
    ref = None
    for i in range(6):
        delta = torch.empty(B * H, T, device=dev)
        d = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
        L().attn_bwd(qd, out, dout, lse, delta, d, B, T, H, D, p, 11,
                     colsum=torch.empty(B * T // 32, 3 * C, device=dev) if i % 2 else None)
        if ref is None:
            ref = d
        else:
            assert torch.equal(d, ref), f"backward {i} differs"


def test_attention_dropout_stats_and_grad_consistency():
    """With p>0 the expected output equals the no-dropout output; the backward regenerates the
    same mask (checked through a finite-difference-free identity: <dO, O> = <dV, V> at fixed P)."""
    B, T, H, D, p = 1, 128, 1, 64, 0.1
    qkv, C = _attn_inputs(B, T, H, 9)
    qd = qkv.to(dev)
    out0 = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    L().attn_fwd(qd, out0, lse, B, T, H, D)
    acc = torch.zeros(B * T, C, device=dev)
    n = 64
    outs = []
    for sd in range(n):
        o = torch.empty_like(out0)
        L().attn_fwd(qd, o, lse, B, T, H, D, p, 1000 + sd)
        acc += o.float()
        outs.append(o)
    assert rel_err((acc / n).cpu(), out0.float().cpu()) < 0.06
    # O is linear in V for fixed mask/P: <dO, O> == <dV, V>
    o = outs[0]
    L().attn_fwd(qd, o, lse, B, T, H, D, p, 1000)
    dout = bf(torch.randn(B * T, C, generator=torch.Generator().manual_seed(10))).to(dev)
    dqkv = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B * H, T, device=dev)
    L().attn_bwd(qd, o, dout, lse, delta, dqkv, B, T, H, D, p, 1000)
    lhs = (dout.float() * o.float()).sum().item()
    rhs = (dqkv[:, 2 * C:].float() * qd[:, 2 * C:].float()).sum().item()
    # the sum cancels heavily: compare against the magnitude of its terms (bf16 dV rounding)
    scale = (dout.float() * o.float()).abs().sum().item()
    assert abs(lhs - rhs) < 2e-3 * scale, (lhs, rhs, scale)


@pytest.mark.parametrize("M,V,ld", [(64, 509, 512), (128, 50257, 50304), (600, 50257, 50432)])
def test_xent(M, V, ld):
    """M = 600 > the row-pipelined kernel's 256 blocks: blocks walk several rows."""
    g = torch.Generator().manual_seed(V + M)
    logits = bf(torch.randn(M, ld, generator=g) * 3)
    labels = torch.randint(0, V, (M,), generator=g)
    labels[3] = -100
    labels[5], labels[7], labels[M - 1] = V - 1, 0, -100  # label in the tail chunk / first column
    lg = logits[:, :V].float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lg, labels, ignore_index=-100)
    ref.backward()
    ld_ = logits.to(dev)
    rows = torch.empty(M, device=dev)
    lse = torch.empty(M, device=dev)
    dl = torch.empty(M, ld, dtype=torch.bfloat16, device=dev)
    loss = torch.empty(1, device=dev)
    inv = torch.empty(1, device=dev)
    L().xent_fwd(ld_, ld, labels.to(dev), rows, lse, dl, ld, M, V, loss, inv)
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, ref.item())
    assert abs(inv.item() - 1.0 / (M - 2)) < 1e-9
    assert rows[3].item() == 0.0 and rows[M - 1].item() == 0.0
    grad = dl.cpu().float()[:, :V] * inv.item()
    assert rel_err(grad, lg.grad) < 4e-3
    assert torch.all(dl[:, V:] == 0)


def test_zero_ranges():
    t = torch.randn(300_000, device=dev)
    ref = t.clone()
    rng = [(0, 1), (5, 1000), (2000, 0), (70_000, 200_001), (299_999, 1)]
    for o, c in rng:
        ref[o:o + c] = 0
    L().zero_ranges(t, torch.tensor(rng, dtype=torch.int64).to(dev))
    torch.cuda.synchronize()
    assert torch.equal(t, ref)


@pytest.mark.parametrize("n", [4096 * 3, 4096 * 3 + 4])  # +4: an odd count of 4-parameter groups (the tail)
def test_adamw_matches_oracle_and_norm(n):
    g = torch.Generator().manual_seed(11)
    p0, gr = torch.randn(n, generator=g), torch.randn(n, generator=g) * 0.01
    params = {"p": p0.clone()}
    state = {}
    pd, gd = p0.to(dev), gr.to(dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    part = torch.empty(L().norm_partials_size(), device=dev)
    gn = torch.empty(1, device=dev)
    for step in (1, 2, 3):
        train_ref.adamw_step(params, {"p": gr}, state, step, lr=1e-3, wd=0.1)
        L().adamw(pd, gd, m, v, pb, n, 1e-3, 0.1, 0.9, 0.95, 1e-8, step, 1.0, part, gn)
    torch.cuda.synchronize()
    assert rel_err(pd.cpu(), params["p"]) < 1e-6
    assert torch.equal(pb.cpu(), bf(pd.cpu()))
    assert abs(gn.item() - gr.norm().item()) < 1e-5 * gr.norm().item()


def test_adamw_in_pieces_with_one_norm_finalisation():
    """FSDP's AdamW (optim.ShardedAdamW): one launch per unit range with grad_norm = NULL, each writing its partial sums
    into its slice of one buffer, then gpt2mi_norm_finalize over all slices: the same parameters as one launch over
    the whole range and the whole range's grad norm."""
    n, cuts = 3 * 4096 + 64, [0, 4096, 4160, 3 * 4096 + 64]
    g = torch.Generator().manual_seed(12)
    p0, gr = torch.randn(n, generator=g).to(dev), (torch.randn(n, generator=g) * 0.01).to(dev)
    P = L().norm_partials_size()
    outs = []
    for pieces in (False, True):
        p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
        gn = torch.empty(1, device=dev)
        part = torch.empty(3 * P, device=dev)
        if pieces:
            for i, (a, b) in enumerate(zip(cuts, cuts[1:])):
                L().adamw(p[a:b], gr[a:b], m[a:b], v[a:b], pb[a:b], b - a, 1e-3, 0.1, 0.9, 0.95, 1e-8, 1, 1.0,
                          part[i * P:(i + 1) * P], None)
            L().norm_finalize(part, 3 * P, gn)
        else:
            L().adamw(p, gr, m, v, pb, n, 1e-3, 0.1, 0.9, 0.95, 1e-8, 1, 1.0, part, gn)
        outs.append((p, pb, gn))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert abs(outs[1][2].item() - gr.norm().item()) < 1e-5 * gr.norm().item()


def test_colsum():
    M, N = 1000, 2304
    g = bf(torch.randn(M, N))
    db = torch.ones(N, device=dev)
    L().colsum_bf16(g.to(dev), db, M, N, N)
    assert rel_err(db.cpu(), 1 + g.float().sum(0)) < 1e-5


@pytest.mark.parametrize("layout,epi", [(0, 0), (0, 2), (0, 3), (1, 0), (1, 4)])
def test_gemm256_matches_gemm128(layout, epi):
    """The ping-pong 256x256, 2-stage 256x256 and 128x128 kernels agree on every fused epilogue (incl.
    dropout)."""
    M, N, K = 320, 768, 192  # partial 256-row tile
    g = torch.Generator().manual_seed(layout * 10 + epi)
    A = bf(torch.randn(M, K, generator=g)).to(dev)
    Bm = bf(torch.randn(N, K, generator=g) if layout == 0 else torch.randn(K, N, generator=g)).to(dev)
    ldb = K if layout == 0 else N
    bias = torch.randn(N, generator=g).to(dev)
    resid = torch.randn(M, N, generator=g).to(dev)
    outs = []
    for impl in (0, 1, 2):
        f32 = epi == 2
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        aux = bf(torch.randn(M, N, generator=torch.Generator().manual_seed(5))).to(dev)
        L().gemm(layout, epi, M, N, K, A, K, Bm, ldb, C, N, bias=bias if layout == 0 else None,
                 resid=resid if epi == 2 else None, aux=aux, ldaux=N, p_drop=0.1, seed=77, sched=impl)
        outs.append((C.float().cpu(), aux.float().cpu()))
    for o in outs[1:]:
        assert rel_err(outs[0][0], o[0]) < 1e-5 if epi == 2 else rel_err(outs[0][0], o[0]) < 2e-3
        assert rel_err(outs[0][1], o[1]) < 2e-3


@pytest.mark.parametrize("M,N,K,splits", [(256, 256, 1024, 1), (512, 768, 4096, 7), (768, 256, 2048, 3),
                                          (768, 512, 4096, 4), (256, 768, 3072, 1)])
def test_gemm_wgrad_splitk_slabs(M, N, K, splits):
    g = torch.Generator().manual_seed(M + N + splits)
    A, B = bf(torch.randn(K, M, generator=g)), bf(torch.randn(K, N, generator=g))
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(dev)
    ws = torch.empty(splits * M * N, device=dev)
    L().gemm_wgrad(M, N, K, A.to(dev), M, B.to(dev), N, C, N, accumulate=True, alpha=0.5, workspace=ws, splits=splits)
    assert rel_err(C.cpu(), C0 + 0.5 * (A.float().t() @ B.float())) < 1e-5
    # deterministic: same inputs -> bitwise same result
    C2 = C0.to(dev)
    L().gemm_wgrad(M, N, K, A.to(dev), M, B.to(dev), N, C2, N, accumulate=True, alpha=0.5, workspace=ws, splits=splits)
    assert torch.equal(C, C2)


@pytest.mark.parametrize("layout", [0, 1])
@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (448, 512, 1024), (256, 2304, 128)])
def test_gemm_pingpong_vs_fp64(layout, M, N, K):
    """The ping-pong kernel (default for N % 256 == 0, even K-tile count) against an fp64 reference:
    full tiles, a partial last row tile, the shortest K (2 K-tiles) and GPT-2 widths."""
    g = torch.Generator().manual_seed(M + N + K + layout)
    A = bf(torch.randn(M, K, generator=g))
    B = bf(torch.randn(N, K, generator=g) if layout == 0 else torch.randn(K, N, generator=g))
    ref = A.double() @ (B.double().t() if layout == 0 else B.double())
    C = torch.full((M, N), 3.0, device=dev)
    L().gemm(layout, L().EPI_F32, M, N, K, A.to(dev), K, B.to(dev), B.shape[1], C, N, alpha=0.25)
    torch.cuda.synchronize()
    assert rel_err(C.cpu(), 0.25 * ref) < 1e-6


@pytest.mark.parametrize("N,epi", [(768, 4), (512, 0), (384, 4)])
def test_gemm_fused_bias_grad(N, epi):
    """dbias[n] += sum_m C[m][n] of the stored bf16 output: fused into the ping-pong epilogue (N % 256 == 0)
    and by a column-sum pass otherwise; same result either way."""
    M, K = 576, 256  # a partial 256-row tile
    g = torch.Generator().manual_seed(N + epi)
    A = bf(torch.randn(M, K, generator=g)).to(dev)
    Bm = bf(torch.randn(K, N, generator=g) * 0.1).to(dev)
    aux = bf(torch.rand(M, N, generator=g)).to(dev)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    db0 = torch.randn(N, generator=g)
    db = db0.to(dev)
    L().gemm(1, epi, M, N, K, A, K, Bm, N, C, N, aux=aux if epi == 4 else None, ldaux=N, dbias=db)
    torch.cuda.synchronize()
    ref = db0.double() + C.cpu().double().sum(0)
    assert rel_err(db.cpu(), ref) < 1e-5


def test_transpose_bf16_batched():
    """Several weights of one arena in one launch (the transposed-shadow refresh) == per-matrix W^T."""
    shapes = [(128, 64), (192, 320), (64, 64), (256, 128)]
    offs, o = [], 0
    for r, c in shapes:
        offs.append(o)
        o += r * c + 64  # gaps stay untouched
    src = bf(torch.randn(o)).to(dev)
    dst = torch.full((o,), 7.0, dtype=torch.bfloat16, device=dev)
    rows, tiles = [], 0
    for (r, c), off in zip(shapes, offs):
        rows.append((off, r, c, tiles))
        tiles += (r // 64) * (c // 64)
    desc = torch.tensor(rows, dtype=torch.int64, device=dev)
    L().transpose_bf16_batched(src, dst, desc, len(rows), tiles)
    torch.cuda.synchronize()
    for (r, c), off in zip(shapes, offs):
        w = src[off:off + r * c].view(r, c)
        assert torch.equal(dst[off:off + r * c].view(c, r), w.t()), (r, c)
        assert torch.all(dst[off + r * c:off + r * c + 64] == 7.0)


@pytest.mark.parametrize("epi", ["plain", "bias", "gelu_drop", "resid_drop", "gelu_bwd_dbias"])
@pytest.mark.parametrize("M,N,K", [(8192, 4096, 768), (65536, 2304, 768), (65536, 768, 768), (65536, 768, 3072),
                                   (16384, 768, 2304)])
def test_gemm_persistent_schedule_bitwise(epi, M, N, K):
    """The persistent ping-pong schedule (short-K forward-layout GEMMs with >= 2 tiles per CU: one block per CU
    walks the tiles, the next tile's first K-tile lands during this tile's epilogue) computes every output
    element exactly as the one-tile-per-block kernel (sched 6 forces that one): bitwise equal,
    and within bf16 rounding of an fp32 reference on sampled rows. Covers every epilogue the step runs on it:
    plain / bias (qkv, proj dgrad), GELU + dropout (fc1), fp32 residual + dropout (proj forward) and the GELU
    derivative product with its fused bias gradient (fc2 dgrad; column sums by atomics, so to fp32 rounding). K = 2304 /
    3072: the long-K shapes the persistent schedule also takes by default (qkv / fc1 dgrad, fc2 + residual)."""
    g = torch.Generator().manual_seed(M + N + K)
    A = bf(torch.randn(M, K, generator=g)).to(dev)
    W = bf(torch.randn(N, K, generator=g) * 0.05).to(dev)
    bias = torch.randn(N, generator=g).to(dev) if epi not in ("plain", "gelu_bwd_dbias") else None
    resid = torch.randn(M, N, generator=g).to(dev) if epi == "resid_drop" else None
    dgelu = bf(torch.rand(M, N, generator=g) * 1.2 - 0.1).to(dev) if epi == "gelu_bwd_dbias" else None
    outs, dbs = [], []
    # SHARED_CUS: the work-queue persistent schedule the data-parallel wrappers take under collectives
    for sched in (L().SCHED_AUTO, 6, L().SCHED_NO_PERSISTENT, L().SCHED_SHARED_CUS):
        C = torch.empty(M, N, dtype=torch.float32 if epi == "resid_drop" else torch.bfloat16, device=dev)
        if epi == "gelu_drop":
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            L().gemm(0, L().EPI_GELU, M, N, K, A, K, W, K, C, N, bias=bias, aux=aux, ldaux=N, p_drop=0.1,
                     seed=99, sched=sched)
            outs.append((C, aux))
        elif epi == "resid_drop":
            L().gemm(0, L().EPI_RESID, M, N, K, A, K, W, K, C, N, bias=bias, resid=resid, p_drop=0.1, seed=98,
                     sched=sched)
            outs.append((C,))
        elif epi == "gelu_bwd_dbias":
            db = torch.zeros(N, device=dev)
            L().gemm(0, L().EPI_GELU_BWD, M, N, K, A, K, W, K, C, N, aux=dgelu, ldaux=N, dbias=db, sched=sched)
            outs.append((C,))
            dbs.append(db)
        else:
            L().gemm(0, L().EPI_BF16, M, N, K, A, K, W, K, C, N, bias=bias, sched=sched)
            outs.append((C,))
    torch.cuda.synchronize()
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)
    rows = torch.arange(0, M, M // 64, device=dev)
    ref = A[rows].float() @ W.float().t() + (bias if bias is not None else 0.0)
    if epi in ("plain", "bias"):
        assert rel_err(outs[0][0][rows].float().cpu(), ref.cpu()) < 4e-3
    if epi == "gelu_bwd_dbias":
        assert rel_err(outs[0][0][rows].float().cpu(), (ref * dgelu[rows].float()).cpu()) < 4e-3
        full = outs[0][0].float().sum(0)  # the bias grad = column sums of the stored (bf16-rounded) output
        for db in dbs:
            assert torch.allclose(db, full, rtol=1e-4, atol=1e-3 * full.abs().max().item())


def test_gemm_work_queue_reuse_across_streams():
    """GPT2MI_SCHED_SHARED_CUS: the persistent GEMM's per-XCD work queues (gemm_pp.hip g_pp_queue, one slot per
    launch over 256 rotating slots, reset by the last block out). 600 launches on two streams wrap the slots twice
    with two grids running at once: every launch covers every tile exactly once (bitwise equal to the static walk),
    so a slot left dirty or shared would show as a missing or doubled tile."""
    M, N, K = 8192, 4096, 768
    g = torch.Generator().manual_seed(5)
    A = bf(torch.randn(M, K, generator=g)).to(dev)
    W = bf(torch.randn(N, K, generator=g) * 0.05).to(dev)
    ref = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, K, A, K, W, K, ref, N, sched=L().SCHED_AUTO)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    bad = 0
    for i in range(600):
        st = streams[i % 2]
        C = outs[i % 4]
        with torch.cuda.stream(st):
            C.fill_(float("nan"))
            L().gemm(0, L().EPI_BF16, M, N, K, A, K, W, K, C, N, sched=L().SCHED_SHARED_CUS)
        if i % 50 == 49:
            torch.cuda.synchronize()
            bad += sum(int(not torch.equal(o, ref)) for o in outs)
    torch.cuda.synchronize()
    assert bad == 0


@pytest.mark.parametrize("m,n,tokens,splits", [(2304, 768, 8192, 4), (768, 3072, 8192, 8), (50432, 768, 4096, 3)])
def test_wgrad_kernels_bitwise(m, n, tokens, splits):
    """The weight gradient on the ping-pong kernel (default) and the 2-stage 256x256 kernel (sched 2): the same K
    order per output element (split counts chosen so both kernels cut K at the same K-tiles), so bitwise equal; and
    within fp32 rounding of a float64 reference on sampled rows."""
    g = torch.Generator().manual_seed(m + n + splits)
    A = bf(torch.randn(tokens, m, generator=g) * 0.1).to(dev)
    B = bf(torch.randn(tokens, n, generator=g)).to(dev)
    ws = torch.empty(splits * m * n, device=dev)
    outs = []
    for impl in (0, 2):
        C = torch.zeros(m, n, device=dev)
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C, n, accumulate=True, workspace=ws, splits=splits, sched=impl)
        outs.append(C)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    rows = torch.arange(0, m, max(1, m // 32), device=dev)
    ref = A[:, rows].double().t() @ B.double()
    err = (outs[0][rows].double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


def _tail(t):
    """t on the device, followed in its allocation by NaN. Since ABI v11 the weight-gradient GEMM's partial-tile reads
    stop at the operand's last element (buffer num_records: lanes past it read zeros), so a NaN there reaches no output,
    stored or not, and no caller needs slack past an operand (the engine allocates its activations without any)."""
    buf = torch.full((t.numel() + 4096,), float("nan"), dtype=t.dtype, device=dev)
    out = buf[:t.numel()].view(t.shape)
    out.copy_(t.to(dev))
    return out


@pytest.mark.parametrize("M,N,K", [(512, 1600, 1600), (256, 4800, 1600), (320, 1600, 4800), (256, 6400, 1600),
                                   (512, 1600, 6400), (64, 64, 128), (256, 320, 192)])
def test_gemm_edge_tiles_and_odd_k_vs_fp64(M, N, K):
    """GPT-2 1.5B's GEMM shapes on the ping-pong kernel: N a multiple of 64 but not of 256 (a partial last column
    tile: 1600 = 6.25 x 256, 4800 = 18.75 x 256) and odd K-tile counts (K = 1600: 25, 4800: 75; run as a zero K-tile
    plus the rest). fp32 output with alpha and accumulate against float64; the columns of a wider C past N stay
    untouched."""
    g = torch.Generator().manual_seed(M + N + K)
    A = bf(torch.randn(M, K, generator=g))
    W = bf(torch.randn(N, K, generator=g))
    C0 = torch.randn(M, N, generator=g)
    ref = C0.double() + 0.25 * (A.double() @ W.double().t())
    ld = N + 64
    C = torch.full((M, ld), 7.0, device=dev)
    C[:, :N] = C0.to(dev)
    L().gemm(0, L().EPI_F32, M, N, K, A.to(dev), K, W.to(dev), K, C, ld, alpha=0.25, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(C[:, :N].cpu(), ref) < 1e-6
    assert torch.all(C[:, N:] == 7.0)


@pytest.mark.parametrize("N,K", [(1600, 1600), (4800, 1600), (1600, 4800)])
def test_gemm_edge_epilogues_vs_oracle(N, K):
    """The fused epilogues the 1.5B step runs on partial column tiles: bias (qkv), fp32 residual + dropout (proj /
    fc2: the oracle's own mask of the site), GELU + dropout with its masked derivative (fc1 at K = 1600), and the
    GELU-derivative product with the fused bias gradient (fc2 dgrad)."""
    from oracle import dropout_ref as D
    M = 512
    g = torch.Generator().manual_seed(N + 3 * K)
    A, W = bf(torch.randn(M, K, generator=g)), bf(torch.randn(N, K, generator=g) * 0.03)
    bias, resid = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    acc = A.double() @ W.double().t()
    Ad, Wd, bd = A.to(dev), W.to(dev), bias.to(dev)
    p, seed = 0.1, (0x8CF69C6F << 32) | 12345
    mask = D.site_scale(seed, M, N, p).double()
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, K, Ad, K, Wd, K, C, N, bias=bd)
    assert rel_err(C.cpu().double(), acc + bias.double()) < 4e-3
    Cr = torch.empty(M, N, device=dev)
    L().gemm(0, L().EPI_RESID, M, N, K, Ad, K, Wd, K, Cr, N, bias=bd, resid=resid.to(dev), p_drop=p, seed=seed)
    assert rel_err(Cr.cpu().double(), resid.double() + (acc + bias.double()) * mask) < 1e-5
    H = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    G = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_GELU, M, N, K, Ad, K, Wd, K, H, N, bias=bd, aux=G, ldaux=N, p_drop=p, seed=seed)
    u = (acc + bias.double()).float().requires_grad_(True)
    (model_ref.gelu_tanh(u) * mask.float()).sum().backward()
    assert rel_err(H.cpu().double(), model_ref.gelu_tanh(u.detach()).double() * mask) < 4e-3
    assert rel_err(G.cpu().double(), u.grad.double()) < 4e-3
    db = torch.zeros(N, device=dev)
    Cg = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_GELU_BWD, M, N, K, Ad, K, Wd, K, Cg, N, aux=G, ldaux=N, dbias=db)
    assert rel_err(Cg.cpu().double(), acc * G.cpu().double()) < 4e-3
    assert rel_err(db.cpu(), Cg.float().sum(0).cpu()) < 1e-4


@pytest.mark.parametrize("m,n,tokens,splits", [(4800, 1600, 4096, 3), (1600, 1600, 2048, 1), (1600, 6400, 2048, 2),
                                               (6400, 1600, 1024, 1), (50432, 1600, 512, 1), (320, 192, 1024, 4)])
def test_gemm_wgrad_edge_tiles_vs_fp64(m, n, tokens, splits):
    """The weight gradients of GPT-2 1.5B (out x in = 4800 x 1600, 1600 x 1600, 1600 x 6400, 6400 x 1600, the tied
    lm_head 50432 x 1600) on the ping-pong kernel with partial last row / column tiles, split-K slabs or one pass,
    write (accumulate=False: the lazy-zeroed arena) and accumulate, against float64 on sampled rows."""
    g = torch.Generator().manual_seed(m + n + tokens)
    A = _tail(bf(torch.randn(tokens, m, generator=g) * 0.1))
    B = _tail(bf(torch.randn(tokens, n, generator=g)))
    ws = torch.empty(max(4, splits * m * n), device=dev)
    C = torch.full((m, n), float("nan"), device=dev)
    L().gemm_wgrad(m, n, tokens, A, m, B, n, C, n, accumulate=False, alpha=0.5, workspace=ws, splits=splits)
    C1 = C.clone()
    L().gemm_wgrad(m, n, tokens, A, m, B, n, C, n, accumulate=True, alpha=0.5, workspace=ws, splits=splits)
    torch.cuda.synchronize()
    rows = torch.cat([torch.arange(0, m, max(1, m // 24), device=dev), torch.arange(m - 8, m, device=dev)])
    ref = 0.5 * (A[:, rows].double().t() @ B.double())
    assert rel_err(C1[rows].double().cpu(), ref.cpu()) < 1e-5
    assert rel_err(C[rows].double().cpu(), 2 * ref.cpu()) < 1e-5
    assert not torch.isnan(C).any()


@pytest.mark.parametrize("m,n,tokens,splits", [(512, 192, 1024, 3), (768, 1600, 2048, 2), (50432, 768, 1024, 3),
                                               (256, 64, 256, 1)])
def test_gemm_wgrad_kt_same_bits_as_wgrad(m, n, tokens, splits):
    """gpt2mi_gemm_wgrad_kt (the X operand given transposed: the tied lm_head's wgrad against lnf^T) against
    gpt2mi_gemm_wgrad on the same operands — the same split-K slabs summed in the same order, so the same bits — with
    write (lazy-zeroed arena) and accumulate, alpha and a device alpha; and against float64 on sampled rows."""
    g = torch.Generator().manual_seed(m + n + tokens + splits)
    A = _tail(bf(torch.randn(tokens, m, generator=g) * 0.1))
    B = _tail(bf(torch.randn(tokens, n, generator=g)))
    Bt = B.t().contiguous()
    ad = torch.tensor([0.75], device=dev)
    ws = torch.empty(max(4, splits * m * n), device=dev)
    C0 = torch.randn(m, n, generator=g).to(dev)
    for acc in (False, True):
        C1, C2 = C0.clone(), C0.clone()
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C1, n, accumulate=acc, alpha=0.5, alpha_dev=ad, workspace=ws,
                       splits=splits)
        L().gemm_wgrad_kt(m, n, tokens, A, m, Bt, tokens, C2, n, accumulate=acc, alpha=0.5, alpha_dev=ad,
                          workspace=ws, splits=splits)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2), (acc, (C1 - C2).abs().max().item())
        rows = torch.cat([torch.arange(0, m, max(1, m // 24), device=dev), torch.arange(m - 8, m, device=dev)])
        ref = 0.375 * (A[:, rows].double().t() @ B.double()) + (C0[rows].double() if acc else 0)
        assert rel_err(C2[rows].double().cpu(), ref.cpu()) < 1e-5


@pytest.mark.parametrize("C,tokens", [(768, 65536), (768, 4096), (1024, 2048), (256, 1024)])
def test_gemm_wgrad_grouped_same_bits_as_wgrad(C, tokens):
    """gpt2mi_gemm_wgrad_grouped (ABI v13: a GPT2Block's qkv / proj / fc1 / fc2 weight gradients as one launch + one
    reduction) against gpt2mi_gemm_wgrad of each problem with the same split-K factor (fp32 slabs): the same bits,
    writing (lazy-zeroed arena) and accumulating, with alpha and a device alpha; sampled rows against float64; at C =
    768 and 65 536 tokens the engine's shapes and split choice."""
    shapes = [(3 * C, C), (C, C), (4 * C, C), (C, 4 * C)]
    sp = L().wgrad_group_splits(shapes, tokens)
    g = torch.Generator(device=dev).manual_seed(C + tokens)
    ops = [((torch.randn(tokens, m, device=dev, generator=g) * 0.05).to(torch.bfloat16),
            torch.randn(tokens, n, device=dev, generator=g).to(torch.bfloat16)) for m, n in shapes]
    ws = torch.empty(sp * sum(m * n for m, n in shapes), device=dev)
    ad = torch.tensor([0.75], device=dev)
    C0 = [torch.randn(m, n, device=dev, generator=g) for m, n in shapes]
    for acc in (False, True):
        Cg = [c.clone() for c in C0]
        probs = [(m, n, A, m, B, n, Cg[i]) for i, ((m, n), (A, B)) in enumerate(zip(shapes, ops))]
        L().gemm_wgrad_grouped(probs, tokens, accumulate=acc, alpha=0.5, alpha_dev=ad, workspace=ws, splits=sp)
        for i, ((m, n), (A, B)) in enumerate(zip(shapes, ops)):
            Ci = C0[i].clone()
            L().gemm_wgrad(m, n, tokens, A, m, B, n, Ci, n, accumulate=acc, alpha=0.5, alpha_dev=ad, workspace=ws,
                           splits=sp)
            torch.cuda.synchronize()
            assert torch.equal(Ci, Cg[i]), (acc, i, (Ci - Cg[i]).abs().max().item())
            rows = torch.cat([torch.arange(0, m, max(1, m // 12), device=dev), torch.arange(m - 4, m, device=dev)])
            ref = 0.375 * (A[:, rows].double().t() @ B.double()) + (C0[i][rows].double() if acc else 0)
            assert rel_err(Cg[i][rows].double().cpu(), ref.cpu()) < 1e-5
    # fewer problems, and the argument checks
    Cg = [c.clone() for c in C0[:2]]
    L().gemm_wgrad_grouped([(m, n, A, m, B, n, Cg[i]) for i, ((m, n), (A, B)) in enumerate(zip(shapes[:2], ops))],
                           tokens, accumulate=False, workspace=ws, splits=sp)
    C1 = torch.empty_like(Cg[1])
    L().gemm_wgrad(shapes[1][0], shapes[1][1], tokens, ops[1][0], shapes[1][0], ops[1][1], shapes[1][1], C1,
                   shapes[1][1], accumulate=False, workspace=ws, splits=sp)
    torch.cuda.synchronize()
    assert torch.equal(C1, Cg[1])
    with pytest.raises(L().KernelError, match="multiples of 256"):
        L().gemm_wgrad_grouped([(192, 256, ops[0][0], 3 * C, ops[0][1], C, Cg[0])], tokens, workspace=ws, splits=sp)
    with pytest.raises(L().KernelError, match="workspace"):
        L().gemm_wgrad_grouped([(m, n, A, m, B, n, c) for (m, n), (A, B), c in zip(shapes, ops, C0)], tokens,
                               workspace=ws[:16], splits=sp)


@pytest.mark.parametrize("m,n", [(50432, 768), (2304, 768), (768, 3072)])
def test_wgrad_full_size_vs_fp64(m, n):
    """The step's weight gradients at BASELINE cfg 2's full size (65 536 tokens, the split-K factor the engine picks)
    against float64 on sampled output rows — the tied lm_head (also through gpt2mi_gemm_wgrad_kt, its transposed-X
    form), qkv and fc2 — not only against each other."""
    tokens = 65536
    sp = L().wgrad_splits(m, n, tokens)
    g = torch.Generator(device=dev).manual_seed(m + n)
    A = (torch.randn(tokens, m, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    B = torch.randn(tokens, n, device=dev, generator=g).to(torch.bfloat16)
    ws = torch.empty(max(4, sp * m * n), device=dev)
    C = torch.empty(m, n, device=dev)
    L().gemm_wgrad(m, n, tokens, A, m, B, n, C, n, accumulate=False, alpha=0.5, workspace=ws, splits=sp)
    rows = torch.cat([torch.arange(0, m, max(1, m // 16), device=dev), torch.arange(m - 4, m, device=dev)])
    ref = 0.5 * (A[:, rows].double().t() @ B.double())
    assert rel_err(C[rows].double().cpu(), ref.cpu()) < 1e-5
    if m % 256 == 0:
        Bt = B.t().contiguous()
        C2 = torch.empty(m, n, device=dev)
        L().gemm_wgrad_kt(m, n, tokens, A, m, Bt, tokens, C2, n, accumulate=False, alpha=0.5, workspace=ws, splits=sp)
        torch.cuda.synchronize()
        assert torch.equal(C, C2)


@pytest.mark.parametrize("m,n,tokens,splits", [(2304, 768, 8192, 4), (768, 3072, 8192, 8), (4800, 1600, 4096, 3),
                                               (1600, 6400, 2048, 2), (50432, 768, 4096, 3), (512, 192, 1024, 1)])
def test_gemm_wgrad_bf16_slabs_vs_fp64(m, n, tokens, splits):
    """GPT2MI_SCHED_BF16_SLABS (the engine's autocast weight gradients): every split-K partial sum rounded once to bf16,
    the slabs summed in fp32 in split order. Against float64: within the error of one bf16 rounding of the sum (the
    reference's autocast wgrad rounds its whole sum to bf16 once, train_gpt2_distributed.py:412), write and accumulate,
    partial last tiles (1.5B widths); deterministic (bitwise on a rerun); the transposed-X form gives the same bits;
    one split (no slabs) gives exactly the fp32-slab path's bits."""
    g = torch.Generator().manual_seed(m + n + tokens + 7 * splits)
    A = _tail(bf(torch.randn(tokens, m, generator=g) * 0.1))
    B = _tail(bf(torch.randn(tokens, n, generator=g)))
    ws = torch.empty(max(4, splits * m * n), device=dev)
    C0 = torch.randn(m, n, generator=g).to(dev)
    f16 = L().SCHED_BF16_SLABS
    rows = torch.cat([torch.arange(0, m, max(1, m // 24), device=dev), torch.arange(m - 8, m, device=dev)])
    ref = 0.5 * (A[:, rows].double().t() @ B.double())
    for acc in (False, True):
        C1, C2, C3 = C0.clone(), C0.clone(), C0.clone()
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C1, n, accumulate=acc, alpha=0.5, workspace=ws, splits=splits,
                       sched=f16)
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C2, n, accumulate=acc, alpha=0.5, workspace=ws, splits=splits,
                       sched=f16)
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C3, n, accumulate=acc, alpha=0.5, workspace=ws, splits=splits)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2)
        want = ref + (C0[rows].double() if acc else 0)
        err = rel_err((C1[rows].double() - (C0[rows].double() if acc else 0)).cpu(), ref.cpu())
        assert err < (1e-5 if splits == 1 else 3e-3), (acc, err)
        assert rel_err(C1[rows].double().cpu(), want.cpu()) < 3e-3
        if splits == 1:
            assert torch.equal(C1, C3)
        if m % 256 == 0:
            Bt = B.t().contiguous()
            C4 = C0.clone()
            L().gemm_wgrad_kt(m, n, tokens, A, m, Bt, tokens, C4, n, accumulate=acc, alpha=0.5, workspace=ws,
                              splits=splits, sched=f16)
            torch.cuda.synchronize()
            assert torch.equal(C1, C4), (acc, (C1 - C4).abs().max().item())


def test_lm_head_dgrad_full_size_vs_fp64():
    """dlnf = dlogits . wte at cfg 2's full size (65 536 x 768 over K = 50 432, the forward layout against the
    transposed wte shadow) against float64 on sampled rows."""
    M, N, Kd = 65536, 768, 50432
    g = torch.Generator(device=dev).manual_seed(5)
    dl = (torch.randn(M, Kd, device=dev, generator=g) * 0.01).to(torch.bfloat16)
    wt = torch.randn(N, Kd, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    L().gemm(0, L().EPI_BF16, M, N, Kd, dl, Kd, wt, Kd, out, N)
    rows = torch.arange(0, M, M // 32, device=dev)
    ref = dl[rows].double() @ wt.double().t()
    assert rel_err(out[rows].double().cpu(), ref.cpu()) < 8e-3


def test_wgrad_slab_precision_per_element_at_the_proj_shape():
    """Per-element error of the weight-gradient split-K slabs at the step's most-split shape: the attention proj
    (768 x 768 over 65 536 tokens, 28 splits), over the elements with |g| below the median (where partial sums cancel).
    Baselines against float64: a single bf16 rounding of the exact sum, and the reference's own autocast weight gradient
    (train_gpt2_distributed.py:404,412: torch.mm of the bf16 operands, fp32 accumulation in hipBLASLt, one rounding to
    bf16). Every fp32 accumulation (the reference's included) loses relative precision on the sums closest to zero, so
    the criterion is taken over median/1000 <= |g| < median: fp32 slabs (the engine's default) within 2x the worst
    single-rounding error there; bf16 slabs (GPT2MI_SCHED_BF16_SLABS, one bf16 rounding per split) are reported, and
    the worst case over ALL below-median elements is reported for every method. Round 4, MI355X: bf16 slabs 488
    (worst, all below-median), fp32 slabs 0.18, single rounding 0.0039 -> fp32 slabs are the default."""
    m = n = 768
    tokens = 65536
    sp = L().wgrad_splits(m, n, tokens)
    assert sp == 28
    g = torch.Generator(device=dev).manual_seed(11)
    A = (torch.randn(tokens, m, device=dev, generator=g) * 1e-3).to(torch.bfloat16)  # dY: a gradient's scale
    B = torch.randn(tokens, n, device=dev, generator=g).to(torch.bfloat16)          # X: a LayerNorm output's
    exact = A.double().t() @ B.double()
    ws = torch.empty(sp * m * n, device=dev)
    out = {}
    for name, sched in (("fp32_slabs", 0), ("bf16_slabs", L().SCHED_BF16_SLABS)):
        C = torch.empty(m, n, device=dev)
        L().gemm_wgrad(m, n, tokens, A, m, B, n, C, n, accumulate=False, workspace=ws, splits=sp, sched=sched)
        out[name] = C.double()
    out["single_bf16_rounding"] = exact.to(torch.bfloat16).double()
    out["reference_autocast_mm"] = torch.mm(A.t(), B).double()
    med = exact.abs().median()
    below = exact.abs() < med
    band = below & (exact.abs() >= med / 1000)
    stats = {}
    for k, v in out.items():
        rel = (v - exact).abs() / exact.abs()
        stats[k] = {"worst_band": rel[band].max().item(), "worst_below_median": rel[below].max().item(),
                    "rms_band": rel[band].pow(2).mean().sqrt().item()}
    print("per-element relative error (band: median/1000 <= |g| < median):", stats)
    bound = 2 * stats["single_bf16_rounding"]["worst_band"]
    assert stats["single_bf16_rounding"]["worst_band"] <= 2 ** -8 * 1.0001
    assert stats["fp32_slabs"]["worst_band"] <= bound, stats
    from gpt_2_distributed_amd.engine import Engine
    default = "bf16_slabs" if Engine.WGRAD_BF16_SLABS else "fp32_slabs"
    assert stats[default]["worst_band"] <= bound, (default, stats)


@pytest.mark.parametrize("n,off", [(1000, 0), (1003, 0), (7_087_872, 0), (4099, 1), (4099, 3)])
def test_fsdp_pack_unpack_accum(n, off):
    """FSDP's flat-unit passes (aux_ops.hip): 8 elements per lane over the 16-B aligned prefix, the element kernels
    over the tail or for unaligned pointers (off = an element offset into the buffers); exactly torch's casts
    (RNE to bf16) and fp32 adds."""
    g = torch.Generator().manual_seed(n + off)
    x = torch.randn(n + off, generator=g).to(dev)
    for dt in (torch.bfloat16, torch.float32):
        # pack: fp32 grad range -> dt, zero-padded to n_pad
        n_pad = n + 37
        packed = torch.full((n_pad + off,), 7.0, dtype=dt, device=dev)
        L().fsdp_pack(x[off:], packed[off:], n, n_pad)
        torch.cuda.synchronize()
        assert torch.equal(packed[off:off + n], x[off:].to(dt)) and bool((packed[off + n:] == 0).all())
        # unpack: dt -> fp32 + bf16 views
        f32 = torch.empty(n + off, device=dev)
        b16 = torch.empty(n + off, dtype=torch.bfloat16, device=dev)
        L().fsdp_unpack(packed[off:], f32[off:], b16[off:], n)
        torch.cuda.synchronize()
        assert torch.equal(f32[off:], packed[off:off + n].float())
        assert torch.equal(b16[off:], packed[off:off + n].float().to(torch.bfloat16))
        # accum: dst (+)= src
        base = torch.randn(n + off, generator=g).to(dev)
        for acc in (True, False):
            d = base.clone()
            L().fsdp_accum(packed[off:], d[off:], n, accumulate=acc)
            torch.cuda.synchronize()
            exp = (base[off:] if acc else 0.0) + packed[off:off + n].float()
            assert torch.equal(d[off:], exp)
