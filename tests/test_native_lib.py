"""The built HIP library loads on a CPU-only host and registers every op
schema (catches schema typos before a GPU run)."""
import glob
import os.path as osp

import pytest
import torch

import deep_graph_matching_consensus_amd as pkg

OPS = ['spmm_csr', 'spmm_csr_out', 'spline_basis', 'dense_masked_softmax',
       'dense_masked_softmax_bwd', 'dense_softmax_transport',
       'dense_softmax_transport_bwd', 'dense_consensus', 'dense_consensus_bwd',
       'topk_dot', 'train_candidates', 'sddmm', 'sparse_consensus_fwd',
       'sparse_consensus_bwd',
       'relu_bias_bwd', 'col_sum', 'reduce_add_rows',
       'gemm_abt', 'piece_plan', 'spmm_pieces_out',
       'sparse_consensus_fwd_prob', 'slot_conv', 'slot_wgrad',
       'slot_wgrad_list', 'adam_multi', 'pack_grads', 'cat_gemm',
       'pair_scores', 'softmax_nll_fwd', 'dense_wgrad', 'fold_weights',
       'slot_compact_plan', 'slot_gemm', 'slot_spmm_rowmap',
       'slot_gather_sum', 'slot_wgrad_f32']


def test_hip_library_registers_all_ops():
    libs = glob.glob(osp.join(osp.dirname(pkg.__file__), '_C_hip*.so'))
    if not libs:
        pytest.skip('HIP extension not built')
    torch.ops.load_library(libs[0])
    for name in OPS:
        op = getattr(torch.ops.dgmc_amd, name)
        assert op.default._schema.name == 'dgmc_amd::' + name
