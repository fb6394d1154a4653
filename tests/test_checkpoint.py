"""Checkpoint schema (reference state-dict keys) and trainer resume."""
import torch

from deep_graph_matching_consensus_amd.datasets import (
    GraphStore, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.models import (DGMC, GIN, RelCNN,
                                                      SplineCNN)
from deep_graph_matching_consensus_amd.train import PairTrainer


def test_reference_state_dict_keys_spline():
    model = DGMC(SplineCNN(1024, 256, 2, 2, cat=False, dropout=0.5),
                 SplineCNN(128, 128, 2, 2, cat=True), num_steps=10)
    sd = model.state_dict()
    expect = {
        'psi_1.convs.0.weight': (25, 1024, 256),
        'psi_1.convs.0.root': (1024, 256),
        'psi_1.convs.0.bias': (256, ),
        'psi_1.convs.0.kernel_size': (2, ),
        'psi_1.convs.0.is_open_spline': (2, ),
        'psi_1.convs.1.weight': (25, 256, 256),
        'psi_1.final.weight': (256, 256),
        'psi_2.convs.0.weight': (25, 128, 128),
        'psi_2.final.weight': (128, 128 + 2 * 128),
        'mlp.0.weight': (128, 128), 'mlp.0.bias': (128, ),
        'mlp.2.weight': (1, 128), 'mlp.2.bias': (1, ),
    }
    for key, shape in expect.items():
        assert tuple(sd[key].shape) == shape, key
    assert sd['psi_1.convs.0.kernel_size'].dtype == torch.long
    assert sd['psi_1.convs.0.is_open_spline'].dtype == torch.uint8
    # Parameter count from SURVEY.md section 2.2 (PascalVOC config).
    n = sum(p.numel() for p in model.parameters())
    assert n == 9504129


def test_reference_state_dict_keys_gin_rel():
    gin = DGMC(GIN(32, 16, 2), GIN(8, 8, 2), num_steps=1).state_dict()
    assert 'psi_1.convs.0.eps' in gin
    assert 'psi_1.convs.0.nn.lins.0.weight' in gin
    assert 'psi_1.convs.0.nn.batch_norms.1.running_var' in gin
    rel_model = DGMC(RelCNN(300, 256, 3, dropout=0.5), RelCNN(32, 32, 3),
                     num_steps=None, k=10)
    rel = rel_model.state_dict()
    for key in ['psi_1.convs.0.lin1.weight', 'psi_1.convs.0.lin2.weight',
                'psi_1.convs.0.root.weight', 'psi_1.convs.0.root.bias',
                'psi_1.batch_norms.2.num_batches_tracked',
                'psi_1.final.weight']:
        assert key in rel, key
    n = sum(p.numel() for p in rel_model.parameters())
    assert n == 914305  # DBP15K parameter total


def test_trainer_checkpoint_resume(tmp_path):
    groups = make_keypoint_datasets(graphs=6, feature_dim=16, seed=5)
    store = GraphStore(groups, 'cpu')

    def make():
        torch.manual_seed(0)
        model = DGMC(SplineCNN(16, 16, 2, 2, cat=False),
                     SplineCNN(8, 8, 2, 2, cat=True), num_steps=1)
        return PairTrainer(model, store, 8, mode='eager', bf16=False,
                           seed=0)

    a = make()
    a.step()
    path = str(tmp_path / 'ckpt.pt')
    a.save(path)
    ref_state = {k: v.clone() for k, v in a.model.state_dict().items()}
    b = make()
    b.load(path)
    assert b.step_count == 1
    for k, v in b.model.state_dict().items():
        assert torch.equal(v, ref_state[k]), k
    sa = a.optimizer.state_dict()['state']
    sb = b.optimizer.state_dict()['state']
    for i in sa:
        assert torch.equal(sa[i]['exp_avg'], sb[i]['exp_avg'])
