"""Exact-fp32 chunked NT GEMM (csrc/hip/gemm_f32.hip): parts read in place
(arbitrary widths % 4, row strides), zero-page tails, bias / ReLU epilogue,
strided output - against fp64, error at most that of torch's fp32 GEMM
(x2) on the same inputs.  Shapes of the DBP15K psi_1 node GEMMs
(/root/reference/dgmc/models/rel.py:28-31,92)."""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import _backend
from deep_graph_matching_consensus_amd.ops import gemm

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('x6', [False, True])
@pytest.mark.parametrize('M,widths,Nn,bias,relu', [
    (19388 + 19572, [300], 768, False, False),     # RelConv layer 0 map
    (39000, [256], 768, False, False),             # layers 1, 2
    (39000, [300, 256, 256, 256], 256, True, False),   # final Linear
    (1000, [4, 132, 64], 64, True, True),          # tails, skinny tiles
    (77, [128], 128, False, True)])
def test_gemm_nt_f32_vs_fp64(M, widths, Nn, bias, relu, x6):
    """Exact-f32 chain and bf16x6 (x6=True, the default arithmetic): max
    error against fp64 at most twice torch's fp32 GEMM's; bf16x6 also at
    most the exact-f32 kernel's."""
    g = torch.Generator(device=DEV).manual_seed(M + Nn)
    # parts as column slices of one wider buffer (strided rows)
    K = sum(widths)
    buf = torch.randn(M, K + 8, device=DEV, generator=g)
    parts, off = [], 0
    for w in widths:
        parts.append(buf[:, off:off + w])
        off += w
    wt = torch.randn(Nn, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(Nn, device=DEV, generator=g) if bias else None
    assert gemm.nt_f32_supported(parts, wt)
    y = gemm.nt_f32(parts, wt, b, relu, x6=x6)
    x = torch.cat(parts, 1)
    ref = x.double() @ wt.double().t()
    y32 = x @ wt.t()
    if bias:
        ref = ref + b.double()
        y32 = y32 + b
    if relu:
        ref, y32 = ref.clamp(min=0), y32.clamp(min=0)
    e = float((y.double() - ref).abs().max())
    e32 = float((y32.double() - ref).abs().max())
    assert e <= 2 * e32 + 1e-7, (e, e32)
    if x6:
        ye = gemm.nt_f32(parts, wt, b, relu, x6=False)
        ee = float((ye.double() - ref).abs().max())
        assert e <= ee, (e, ee)
        # the scheduled-split variant: same products, same order
        assert torch.equal(gemm.nt_f32(parts, wt, b, relu, x6=True, sched=1),
                           y)


def test_gemm_nt_f32_out_view_and_linear_parts():
    """``out=`` writes a column slice of a larger buffer; linear_parts (the
    RelCNN head) equals F.linear on the concatenation, gradients included."""
    g = torch.Generator(device=DEV).manual_seed(1)
    a = torch.randn(500, 300, device=DEV, generator=g)
    w = torch.randn(128, 300, device=DEV, generator=g) / 17
    big = torch.full((500, 256), 7.0, device=DEV)
    _backend.ops().gemm_nt_f32([a], w, None, False, big[:, 64:192])
    torch.testing.assert_close(big[:, 64:192], a @ w.t(), rtol=1e-5,
                               atol=1e-5)
    assert bool((big[:, :64] == 7).all() and (big[:, 192:] == 7).all())
    lin = torch.nn.Linear(300 + 256, 256).to(DEV)
    h = torch.randn(500, 256, device=DEV, generator=g, requires_grad=True)
    a.requires_grad_()
    y = gemm.linear_parts([a, h], lin.weight, lin.bias)
    ref = torch.nn.functional.linear(torch.cat([a, h], 1), lin.weight,
                                     lin.bias)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    go = torch.randn_like(y)
    g1 = torch.autograd.grad(y, [a, h, lin.weight, lin.bias], go)
    g2 = torch.autograd.grad(ref, [a, h, lin.weight, lin.bias], go)
    for u, v in zip(g1, g2):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('M,cin,cout,bias', [(2000, 128, 256, True),
                                             (777, 64, 64, False),
                                             (4096, 300, 128, True)])
def test_linear_fp32_on_native_nt_gemm(M, cin, cout, bias):
    """``ops.gemm.linear`` (GIN / MLP / encoder Linears, /root/reference/
    dgmc/models/gin.py:49, mlp.py:35): fp32 forward on the exact-f32 NT
    kernel, gradients equal F.linear's to fp32 tolerance."""
    g = torch.Generator(device=DEV).manual_seed(M + cin)
    lin = torch.nn.Linear(cin, cout, bias=bias).to(DEV)
    x = torch.randn(M, cin, device=DEV, generator=g, requires_grad=True)
    wt = lin.weight.detach().t().t()
    assert gemm.nt_f32_supported([x.detach()], wt.contiguous())
    y = gemm.linear(x, lin.weight, lin.bias)
    ref = torch.nn.functional.linear(x, lin.weight, lin.bias)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    go = torch.randn_like(y)
    leaves = [x, lin.weight] + ([lin.bias] if bias else [])
    g1 = torch.autograd.grad(y, leaves, go)
    g2 = torch.autograd.grad(ref, leaves, go)
    # (weight gradients sum M products: fp32 order noise scales with |dW|)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-4,
                                   atol=1e-5 * max(1.0, float(b.abs().max())))


@pytest.mark.parametrize('seed', [0, 1, 2])
@pytest.mark.parametrize('case', ['wide', 'cancel', 'relu'])
def test_gemm_nt_x6_stress_vs_exact(case, seed):
    """The bf16x6 chunked GEMM on the inputs of tests/test_x6_stress.py's
    gate (DBP15K map shape, 300 -> 256): per-row error relative to the row's
    largest fp64 value, at most the exact-f32 chain's."""
    g = torch.Generator(device=DEV).manual_seed(100 + seed)
    M, K, Nn = 4096, 300, 256
    x = torch.randn(M, K, device=DEV, generator=g)
    w = torch.randn(Nn, K, device=DEV, generator=g) / K ** 0.5
    if case == 'wide':
        e = torch.randint(-30, 31, (M, 1), device=DEV, generator=g)
        x = x * torch.pow(2.0, e.float())
    elif case == 'cancel':
        h = K // 2
        x[:, h:2 * h] = x[:, :h]
        w[:, h:2 * h] = -w[:, :h] * (1 + 1e-3 * torch.randn(
            Nn, h, device=DEV, generator=g))
    else:
        x = torch.relu(x - 0.2)
    ref = x.double() @ w.double().t()
    scale = ref.abs().amax(1, keepdim=True).clamp_min(1e-300)
    errs = []
    for x6 in (True, False):
        y = gemm.nt_f32([x], w, None, False, x6=x6)
        errs.append(float(((y.double() - ref).abs() / scale).amax()))
    assert errs[0] <= errs[1], errs
