"""Synthetic dataset generators: shapes and collation semantics."""
import torch

from deep_graph_matching_consensus_amd.datasets import (
    PASCAL_VOC_CATEGORIES, WILLOW_CATEGORIES, make_keypoint_datasets)
from deep_graph_matching_consensus_amd.datasets.kg import make_kg_pair
from deep_graph_matching_consensus_amd.datasets.random_graphs import (
    RandomGraphDataset, make_er_pair, pascal_pf_transform)
from deep_graph_matching_consensus_amd.graph import DataLoader


def test_keypoint_datasets_shape():
    groups = make_keypoint_datasets(PASCAL_VOC_CATEGORIES, graphs=4,
                                    feature_dim=16)
    assert len(groups) == 20
    for (name, K), ds in zip(PASCAL_VOC_CATEGORIES, groups):
        for g in ds:
            assert g.num_nodes <= K and g.y.max() < K
            assert g.edge_attr.min() >= 0 and g.edge_attr.max() <= 1
            assert g.edge_index.size(1) == g.edge_attr.size(0)
    willow = make_keypoint_datasets(WILLOW_CATEGORIES, graphs=3,
                                    visible_prob=1.0, feature_dim=8)
    assert all(g.num_nodes == 10 for ds in willow for g in ds)


def test_pascal_pf_collation_offsets():
    torch.manual_seed(0)
    ds = RandomGraphDataset(5, 8, 0, 3, transform=pascal_pf_transform())
    batch = next(iter(DataLoader(ds, 4, follow_batch=['x_s', 'x_t'])))
    # y_index_s becomes a global source row, y_t stays a local column
    assert batch.y_index_s.max() < batch.x_s.size(0)
    assert batch.y_t.max() < 8
    assert batch.x_s.size(1) == 1 and batch.edge_attr_s.size(1) == 2
    assert batch.edge_index_s.max() < batch.x_s.size(0)


def test_er_pair_permutation():
    s, t, y = make_er_pair(20, 0.3, seed=1)
    assert sorted(y[1].tolist()) == list(range(20))
    assert s.edge_index.size(0) == 2 and t.edge_index.max() < 20


def test_kg_pair_sizes():
    d = make_kg_pair('zh_en', scale=0.05, seed=0)
    assert d.x1.size(1) == 300 and d.x2.size(1) == 300
    n = d.train_y.size(1) + d.test_y.size(1)
    assert n == int(15000 * 0.05)
    assert d.train_y[0].max() < d.x1.size(0)
    assert d.train_y[1].max() < d.x2.size(0)


def test_cli_presets_list_and_er_train(capsys):
    from deep_graph_matching_consensus_amd import cli
    assert cli.main(['list']) == 0
    out = capsys.readouterr().out
    for name in ('er', 'willow', 'pascal', 'pascal_pf', 'dbp15k'):
        assert name in out


def test_cli_info_reports_build_state(capsys, tmp_path):
    import json
    from deep_graph_matching_consensus_amd import cli
    assert cli.main(['info', '--json']) == 0
    rep = json.loads(capsys.readouterr().out)
    for key in ('torch', 'gpu', 'libraries', 'ops', 'build', 'switches'):
        assert key in rep
    assert rep['libraries']['host']['loaded']
    # build_status against a synthetic tree: one edited, one new source
    src = tmp_path / 'csrc' / 'hip'
    src.mkdir(parents=True)
    (src / 'a.hip').write_text('a')
    (src / 'b.hip').write_text('b')
    (tmp_path / 'lib.so').write_text('x')
    man = {'arch': 'gfx950',
           'sources': {'csrc/hip/a.hip': cli._sha256(str(src / 'a.hip')),
                       'csrc/hip/b.hip': 'old'},
           'libraries': {'lib.so': cli._sha256(str(tmp_path / 'lib.so'))}}
    (tmp_path / 'build' / 'native').mkdir(parents=True)
    (tmp_path / 'build' / 'native' / 'manifest.json').write_text(
        json.dumps(man))
    (src / 'c.hip').write_text('c')
    st = cli.build_status(str(tmp_path))
    assert st['manifest'] and st['arch'] == 'gfx950'
    assert st['stale_sources'] == ['csrc/hip/b.hip', 'csrc/hip/c.hip']
    assert st['changed_libs'] == []
    (tmp_path / 'lib.so').write_text('y')
    assert cli.build_status(str(tmp_path))['changed_libs'] == ['lib.so']
