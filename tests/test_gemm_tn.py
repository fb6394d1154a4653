"""Split-K TN GEMM (csrc/hip/gemm_tn.hip) and the generic-width NT GEMM
(csrc/hip/gemm_f32.hip: masked last column block, beta = 1 epilogue): the
weight / input gradients of RelConv's stacked map and of the encoders'
final Linear (/root/reference/dgmc/models/rel.py:28-31,92), GIN / MLP
Linears (gin.py:49, mlp.py:35) - against fp64, error at most twice that of
torch's fp32 product on the same inputs; and the DBP15K psi_1 training
backward without any library (hipBLASLt / rocBLAS) GEMM."""
import pytest
import torch

from deep_graph_matching_consensus_amd.ops import gemm

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _parts(K, widths, g, pad=8, scale=1.0):
    """Column slices of one wider buffer (strided rows)."""
    buf = torch.randn(K, sum(widths) + pad, device=DEV, generator=g) * scale
    out, off = [], 0
    for w in widths:
        out.append(buf[:, off:off + w])
        off += w
    return out


@pytest.mark.parametrize('x6', [True, False])
@pytest.mark.parametrize('K,wa,wb', [
    (38960, [768], [300]),                 # RelConv layer 0 weight gradient
    (38960, [768], [256]),                 # layers 1, 2
    (38960, [256], [300, 256, 256, 256]),  # final Linear on [x | h1 | h2 | h3]
    (1000, [36, 4], [12, 132]),            # narrow parts, partial tiles
    (77, [128], [128]),                    # K below one split step
    (5, [4], [8])])
def test_gemm_tn_vs_fp64(K, wa, wb, x6):
    g = torch.Generator(device=DEV).manual_seed(K + sum(wa) + sum(wb))
    a = _parts(K, wa, g)
    b = _parts(K, wb, g, scale=0.1)
    assert gemm.tn_f32_supported(a, b)
    y = gemm.tn_f32(a, b, x6=x6)
    A, B = torch.cat(a, 1), torch.cat(b, 1)
    ref = A.double().t() @ B.double()
    y32 = A.t() @ B
    assert y.shape == ref.shape
    e = float((y.double() - ref).abs().max())
    e32 = float((y32.double() - ref).abs().max())
    assert e <= 2 * e32 + 1e-6, (e, e32)
    if x6:
        ye = gemm.tn_f32(a, b, x6=False)
        ee = float((ye.double() - ref).abs().max())
        assert e <= 1.5 * ee + 1e-6, (e, ee)
        # every staging variant: the same products per element, in the same
        # k order - bit-identical results
        for cfg in (1, 2, 4):
            yc = gemm.tn_f32(a, b, x6=True, cfg=cfg)
            assert torch.equal(yc, y), (cfg, float((yc - y).abs().max()),
                                        float((yc.double() - ref).abs()
                                              .max()), e)


def test_gemm_tn_accumulate_into_strided_out_and_determinism():
    g = torch.Generator(device=DEV).manual_seed(3)
    a = _parts(5000, [256], g)
    b = _parts(5000, [300], g)
    big = torch.randn(256, 400, device=DEV, generator=g)
    before = big.clone()
    view = big[:, 50:350]
    gemm.tn_f32(a, b, out=view, accumulate=True)
    ref = before[:, 50:350].double() + a[0].double().t() @ b[0].double()
    torch.testing.assert_close(view.double(), ref, rtol=1e-5, atol=1e-4)
    assert torch.equal(big[:, :50], before[:, :50])
    assert torch.equal(big[:, 350:], before[:, 350:])
    # fixed-order fold: bit-identical across runs
    y1 = gemm.tn_f32(a, b)
    y2 = gemm.tn_f32(a, b)
    assert torch.equal(y1, y2)


@pytest.mark.parametrize('x6', [True, False])
@pytest.mark.parametrize('Nn,bias,relu', [(300, True, False),
                                          (36, False, True),
                                          (1068, True, True)])
def test_gemm_nt_masked_columns_and_accumulate(Nn, bias, relu, x6):
    """Output widths that are not multiples of the tile (masked last column
    block, bias read masked) and beta = 1 into a column slice."""
    g = torch.Generator(device=DEV).manual_seed(Nn)
    M, K = 3000, 256
    x = torch.randn(M, K, device=DEV, generator=g)
    wt = torch.randn(Nn, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(Nn, device=DEV, generator=g) if bias else None
    assert gemm.nt_f32_supported([x], wt)
    y = gemm.nt_f32([x], wt, b, relu, x6=x6)
    ref = x.double() @ wt.double().t()
    y32 = x @ wt.t()
    if bias:
        ref, y32 = ref + b.double(), y32 + b
    if relu:
        ref, y32 = ref.clamp(min=0), y32.clamp(min=0)
    e = float((y.double() - ref).abs().max())
    e32 = float((y32.double() - ref).abs().max())
    assert e <= 2 * e32 + 1e-7, (e, e32)
    big = torch.randn(M, Nn + 64, device=DEV, generator=g)
    before = big.clone()
    gemm.nt_f32([x], wt, None, False, out=big[:, 32:32 + Nn], x6=x6,
                accumulate=True)
    torch.testing.assert_close(
        big[:, 32:32 + Nn].double(),
        before[:, 32:32 + Nn].double() + x.double() @ wt.double().t(),
        rtol=1e-5, atol=1e-4)
    assert torch.equal(big[:, :32], before[:, :32])
    assert torch.equal(big[:, 32 + Nn:], before[:, 32 + Nn:])


def _library_gemms(fn):
    """Names of hipBLASLt / rocBLAS kernels launched by ``fn()``."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events()}
    return sorted(n for n in names
                  if n.startswith('Cijk') or 'rocblas' in n.lower() or
                  'hipblaslt' in n.lower())


def test_rel_cnn_psi1_training_backward_native_vs_fp64():
    """psi_1 = RelCNN(300, 256, 3, cat, lin) of the DBP15K config
    (/root/reference/examples/dbp15k.py:29-31; dropout 0 for a
    deterministic comparison) on a KG-shaped graph: forward and every
    parameter gradient against the fp64 reference expression (reference
    mode, ATen ops), error at most 4x the fp32 reference expression's - and
    no library GEMM anywhere in forward + backward."""
    from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
    from deep_graph_matching_consensus_amd.models import RelCNN
    from deep_graph_matching_consensus_amd.runtime import reference_mode
    data = make_kg_pair('zh_en', scale=0.25, seed=0).to(DEV)
    x = torch.cat([data.x1, data.x2], 0)
    n1 = data.x1.size(0)
    ei = torch.cat([data.edge_index1, data.edge_index2 + n1], 1)
    torch.manual_seed(0)
    model = RelCNN(x.size(1), 256, 3, batch_norm=False, cat=True, lin=True,
                   dropout=0.0).to(DEV)
    go = torch.randn(x.size(0), 256, device=DEV)
    # (batch_norm=False: the always-built BatchNorm modules take no part)
    names = [n for n, _ in model.named_parameters()
             if not n.startswith('batch_norms')]
    params = [dict(model.named_parameters())[n] for n in names]

    def run():
        out = model(x, ei)
        return out, torch.autograd.grad(out, params, go)

    assert _library_gemms(run) == []
    out, grads = run()

    def oracle(dtype):
        m2 = RelCNN(x.size(1), 256, 3, batch_norm=False, cat=True, lin=True,
                    dropout=0.0).to(DEV).to(dtype)
        m2.load_state_dict({k: v.to(dtype)
                            for k, v in model.state_dict().items()})
        with reference_mode(True):
            o = m2(x.to(dtype), ei)
            p2 = dict(m2.named_parameters())
            gs = torch.autograd.grad(o, [p2[n] for n in names], go.to(dtype))
        return o, gs

    o64, g64 = oracle(torch.float64)
    o32, g32 = oracle(torch.float32)

    bad = []

    def check(a, b32, b64, what):
        e = float((a.detach().double() - b64).abs().max())
        e32 = float((b32.double() - b64).abs().max())
        if not e <= 4 * e32 + 1e-6 * float(b64.abs().max()):
            bad.append((what, e, e32))

    check(out, o32, o64, 'out')
    for n, a, b32, b64 in zip(names, grads, g32, g64):
        check(a, b32, b64, n)
    assert not bad, bad
