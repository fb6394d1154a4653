"""Run-twice bitwise determinism of the full training step on the GPU (no
float atomics anywhere: SpMM, column reductions, split-K combines and the
consensus kernels all reduce in a fixed order)."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets import (
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import DGMC, SplineCNN
from deep_graph_matching_consensus_amd.train import PairTrainer

pytestmark = pytest.mark.gpu


def _run(mode, steps=3):
    groups = make_keypoint_datasets(graphs=16, feature_dim=64, seed=7)
    store = GraphStore(groups, 'cuda')
    torch.manual_seed(0)
    torch.cuda.manual_seed(0)
    model = DGMC(SplineCNN(64, 64, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(32, 32, 2, 2, cat=True), num_steps=4).cuda()
    tr = PairTrainer(model, store, 32, mode=mode, bf16=True, seed=0)
    torch.manual_seed(1)
    torch.cuda.manual_seed(1)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return tr.read_stats(), {k: v.detach().clone()
                             for k, v in model.state_dict().items()}


@pytest.mark.parametrize('mode', ['eager', 'graph'])
def test_training_is_bitwise_deterministic(mode):
    s1, p1 = _run(mode)
    s2, p2 = _run(mode)
    assert s1['loss_sum'] == s2['loss_sum']
    for k in p1:
        assert torch.equal(p1[k], p2[k]), k


def _run_flagship(bf16, mode='graph', steps=3, buckets=True):
    """Flagship-shaped psi_2 (128 -> 128): bf16 = fused slot conv and
    loop-folded slot weight gradients; fp32 = the used-pair slot GEMMs
    (ops/slot_gemm.py) - in the captured step."""
    groups = make_keypoint_datasets(graphs=16, feature_dim=128, seed=7)
    store = GraphStore(groups, 'cuda',
                       x_dtype=torch.bfloat16 if bf16 else torch.float32)
    torch.manual_seed(0)
    torch.cuda.manual_seed(0)
    model = DGMC(SplineCNN(128, 128, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=4).cuda()
    tr = PairTrainer(model, store, 32, mode=mode, bf16=bf16, seed=0,
                     buckets=buckets)
    torch.manual_seed(1)
    torch.cuda.manual_seed(1)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return tr.read_stats(), {k: v.detach().clone()
                             for k, v in model.state_dict().items()}


@pytest.mark.parametrize('bf16', [True, False])
def test_flagship_step_is_bitwise_deterministic(bf16):
    s1, p1 = _run_flagship(bf16)
    s0, p0 = _run_flagship(bf16)
    assert s1['loss_sum'] == s0['loss_sum']
    for k in p1:
        assert torch.equal(p1[k], p0[k]), k


def test_fp32_graph_step_matches_static_step():
    """Reference precision: the captured step follows the same trajectory as
    the step run eagerly on the same static batches - the capture warm-ups
    (8 real steps) are undone.  (Kernels differ only in fp32 summation
    order across captured / uncaptured launches.)"""
    sg, pg = _run_flagship(False, 'graph', buckets=False)
    ss, ps = _run_flagship(False, 'static')
    assert abs(sg['loss_sum'] - ss['loss_sum']) <= 1e-4 * abs(ss['loss_sum'])
    for k in pg:
        torch.testing.assert_close(pg[k], ps[k], atol=1e-4, rtol=1e-3)
