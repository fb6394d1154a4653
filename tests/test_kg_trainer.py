"""KGTrainer (DBP15K driver semantics, reference examples/dbp15k.py:37-69):
two-phase schedule, psi_1 frozen by ``detach`` in the refinement phase,
Hits@k evaluation - on the CPU (eager) and, marked ``gpu``, with each phase
captured in a hipGraph on the HIP kernels."""
import pytest
import torch

from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
from deep_graph_matching_consensus_amd.models import DGMC, RelCNN
from deep_graph_matching_consensus_amd.train import KGTrainer


def _setup(device, scale=0.02):
    torch.manual_seed(0)
    data = make_kg_pair('zh_en', scale=scale, feature_dim=32,
                        seed=0).to(device)
    psi_1 = RelCNN(data.x1.size(-1), 32, 2, batch_norm=False, cat=True,
                   lin=True, dropout=0.5)
    psi_2 = RelCNN(8, 8, 2, batch_norm=False, cat=True, lin=True)
    model = DGMC(psi_1, psi_2, num_steps=None, k=5).to(device)
    return data, model


def _run_schedule(device, graph):
    data, model = _setup(device)
    trainer = KGTrainer(model, data, lr=1e-2, graph=graph)
    psi_1 = {n: p.detach().clone() for n, p in model.psi_1.named_parameters()}
    model.num_steps, model.detach = 0, False          # phase 1
    for _ in range(3):
        trainer.step()
    loss1 = float(trainer.last_loss)
    moved = [n for n, p in model.psi_1.named_parameters()
             if not torch.equal(p.detach(), psi_1[n])]
    assert moved, 'phase 1 must train psi_1'
    psi_1 = {n: p.detach().clone() for n, p in model.psi_1.named_parameters()}
    mlp = [p.detach().clone() for p in model.mlp.parameters()]
    model.num_steps, model.detach = 2, True           # phase 2
    for _ in range(3):
        trainer.step()
    loss2 = float(trainer.last_loss)
    # detach: psi_1 receives no gradient, so Adam leaves it untouched (the
    # captured step lets autograd steal gradients; None grads are skipped).
    for n, p in model.psi_1.named_parameters():
        assert torch.equal(p.detach(), psi_1[n]), n
    assert any(not torch.equal(p.detach(), q)
               for p, q in zip(model.mlp.parameters(), mlp))
    assert torch.isfinite(torch.tensor([loss1, loss2])).all()
    hits1, hits10 = trainer.evaluate(k=10)
    assert 0.0 <= hits1 <= hits10 <= 1.0
    return loss1, loss2


def test_kg_trainer_two_phase_cpu():
    _run_schedule(torch.device('cpu'), graph=False)


@pytest.mark.gpu
def test_kg_trainer_two_phase_graph_captured_gpu():
    from deep_graph_matching_consensus_amd.ops import _backend
    assert _backend.hip_available()
    _run_schedule(torch.device('cuda'), graph=True)


def _guard_case(device, graph):
    data, model = _setup(device)
    trainer = KGTrainer(model, data, lr=1e-2, graph=graph)
    model.num_steps, model.detach = 0, False
    trainer.step()
    before = [p.detach().clone() for p in model.parameters()]
    x = data.x1.clone()
    data.x1[0, 0] = float("nan")     # in place: the captured step reads it
    trainer.step()
    assert float(trainer.skipped) == 1.0
    for p, q in zip(model.parameters(), before):
        assert torch.equal(p.detach(), q), 'a non-finite step must not update'
    data.x1.copy_(x)
    trainer.step()
    assert float(trainer.skipped) == 1.0
    assert any(not torch.equal(p.detach(), q)
               for p, q in zip(model.parameters(), before))


def test_kg_trainer_nonfinite_guard_cpu():
    _guard_case(torch.device('cpu'), graph=False)


@pytest.mark.gpu
def test_kg_trainer_nonfinite_guard_graph_gpu():
    from deep_graph_matching_consensus_amd.runtime import optim as hip_optim
    data, model = _setup(torch.device('cuda'))
    trainer = KGTrainer(model, data, lr=1e-2, graph=True)
    assert hip_optim.supported(trainer.optimizer)
    _guard_case(torch.device('cuda'), graph=True)


@pytest.mark.gpu
def test_kg_trainer_hip_adam_matches_torch_adam():
    """KGTrainer's HIP multi-tensor Adam follows torch's Adam (eager)."""
    from deep_graph_matching_consensus_amd.runtime import optim as hip_optim
    params = {}
    for enabled in (True, False):
        hip_optim.ENABLED = enabled
        try:
            data, model = _setup(torch.device('cuda'))
            trainer = KGTrainer(model, data, lr=1e-2, graph=False)
            model.num_steps, model.detach = 0, False
            for _ in range(3):
                trainer.step()
        finally:
            hip_optim.ENABLED = True
        params[enabled] = [p.detach().cpu() for p in model.parameters()]
    for a, b in zip(params[True], params[False]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)
