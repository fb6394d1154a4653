// Host-side pair collation (native data loader core).
//
// The reference collates graph pairs in Python (PyG Batch.from_data_list with
// the PairData.__inc__ rule, /root/reference/dgmc/utils/data.py:9-16, and
// follow_batch=['x_s', 'x_t'] in examples/pascal.py:42-43).  For the
// MI355X pipeline the whole synthetic dataset stays resident in HBM; per step
// the host only decides WHICH graphs form the batch and emits compact int64
// index arrays (node/edge gather lists, offset edge_index, batch vectors,
// per-graph counts, ground truth).  The device then gathers features with a
// handful of index_select kernels.  OpenMP parallelises over pairs.
#include <torch/library.h>
#include <ATen/ATen.h>

#include <cstdint>
#include <vector>

namespace dgmc_host {

using at::Tensor;

static void check_cpu_long(const Tensor& t, const char* name) {
  TORCH_CHECK(!t.is_cuda() && t.scalar_type() == at::kLong && t.is_contiguous(),
              name, " must be a contiguous int64 CPU tensor");
}

// Returns (node_idx_s, node_idx_t, edge_idx_s, edge_idx_t, edge_index_s,
//          edge_index_t, batch_s, batch_t, counts_s, counts_t, y)
std::vector<Tensor> collate_pairs(const Tensor& node_ptr, const Tensor& edge_ptr,
                                  const Tensor& edge_local,
                                  const Tensor& node_class,
                                  const Tensor& pos_of_class,
                                  const Tensor& s_ids, const Tensor& t_ids) {
  check_cpu_long(node_ptr, "node_ptr");
  check_cpu_long(edge_ptr, "edge_ptr");
  check_cpu_long(edge_local, "edge_local");
  check_cpu_long(node_class, "node_class");
  check_cpu_long(pos_of_class, "pos_of_class");
  check_cpu_long(s_ids, "s_ids");
  check_cpu_long(t_ids, "t_ids");
  TORCH_CHECK(edge_local.dim() == 2 && edge_local.size(0) == 2, "edge_local");
  const int64_t B = s_ids.numel();
  TORCH_CHECK(t_ids.numel() == B, "s_ids / t_ids size mismatch");
  const int64_t G = node_ptr.numel() - 1;
  const int64_t C = pos_of_class.dim() == 2 ? pos_of_class.size(1) : 0;
  const int64_t E_all = edge_local.size(1);
  const int64_t* np_ = node_ptr.data_ptr<int64_t>();
  const int64_t* ep_ = edge_ptr.data_ptr<int64_t>();
  const int64_t* src_ = edge_local.data_ptr<int64_t>();
  const int64_t* dst_ = src_ + E_all;
  const int64_t* cls_ = node_class.data_ptr<int64_t>();
  const int64_t* poc_ = pos_of_class.data_ptr<int64_t>();
  const int64_t* sid = s_ids.data_ptr<int64_t>();
  const int64_t* tid = t_ids.data_ptr<int64_t>();

  // Exclusive scans of node / edge counts per pair (serial: B is small).
  std::vector<int64_t> ns_off(B + 1, 0), nt_off(B + 1, 0), es_off(B + 1, 0),
      et_off(B + 1, 0);
  for (int64_t b = 0; b < B; ++b) {
    const int64_t gs = sid[b], gt = tid[b];
    TORCH_CHECK(gs >= 0 && gs < G && gt >= 0 && gt < G, "graph id out of range");
    ns_off[b + 1] = ns_off[b] + (np_[gs + 1] - np_[gs]);
    nt_off[b + 1] = nt_off[b] + (np_[gt + 1] - np_[gt]);
    es_off[b + 1] = es_off[b] + (ep_[gs + 1] - ep_[gs]);
    et_off[b + 1] = et_off[b] + (ep_[gt + 1] - ep_[gt]);
  }
  auto L = at::TensorOptions().dtype(at::kLong);
  Tensor node_idx_s = at::empty({ns_off[B]}, L), node_idx_t = at::empty({nt_off[B]}, L);
  Tensor edge_idx_s = at::empty({es_off[B]}, L), edge_idx_t = at::empty({et_off[B]}, L);
  Tensor ei_s = at::empty({2, es_off[B]}, L), ei_t = at::empty({2, et_off[B]}, L);
  Tensor batch_s = at::empty({ns_off[B]}, L), batch_t = at::empty({nt_off[B]}, L);
  Tensor counts_s = at::empty({B}, L), counts_t = at::empty({B}, L);
  Tensor y = at::empty({ns_off[B]}, L);
  int64_t *nis = node_idx_s.data_ptr<int64_t>(), *nit = node_idx_t.data_ptr<int64_t>();
  int64_t *eis = edge_idx_s.data_ptr<int64_t>(), *eit = edge_idx_t.data_ptr<int64_t>();
  int64_t *eis0 = ei_s.data_ptr<int64_t>(), *eis1 = eis0 + es_off[B];
  int64_t *eit0 = ei_t.data_ptr<int64_t>(), *eit1 = eit0 + et_off[B];
  int64_t *bs = batch_s.data_ptr<int64_t>(), *bt = batch_t.data_ptr<int64_t>();
  int64_t *cs = counts_s.data_ptr<int64_t>(), *ct = counts_t.data_ptr<int64_t>();
  int64_t* yp = y.data_ptr<int64_t>();

#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    const int64_t gs = sid[b], gt = tid[b];
    const int64_t n0s = np_[gs], nns = np_[gs + 1] - n0s;
    const int64_t n0t = np_[gt], nnt = np_[gt + 1] - n0t;
    cs[b] = nns;
    ct[b] = nnt;
    for (int64_t i = 0; i < nns; ++i) {
      nis[ns_off[b] + i] = n0s + i;
      bs[ns_off[b] + i] = b;
      const int64_t c = cls_[n0s + i];
      yp[ns_off[b] + i] = (c >= 0 && c < C) ? poc_[gt * C + c] : -1;
    }
    for (int64_t i = 0; i < nnt; ++i) {
      nit[nt_off[b] + i] = n0t + i;
      bt[nt_off[b] + i] = b;
    }
    const int64_t e0s = ep_[gs], nes = ep_[gs + 1] - e0s;
    for (int64_t e = 0; e < nes; ++e) {
      const int64_t o = es_off[b] + e;
      eis[o] = e0s + e;
      eis0[o] = src_[e0s + e] + ns_off[b];
      eis1[o] = dst_[e0s + e] + ns_off[b];
    }
    const int64_t e0t = ep_[gt], net = ep_[gt + 1] - e0t;
    for (int64_t e = 0; e < net; ++e) {
      const int64_t o = et_off[b] + e;
      eit[o] = e0t + e;
      eit0[o] = src_[e0t + e] + nt_off[b];
      eit1[o] = dst_[e0t + e] + nt_off[b];
    }
  }
  return {node_idx_s, node_idx_t, edge_idx_s, edge_idx_t, ei_s, ei_t,
          batch_s,    batch_t,    counts_s,   counts_t,   y};
}

// Static-shape variant for hipGraph replay: writes every index array of the
// batch, padded to fixed capacities, into ONE preallocated (pinned) int64
// buffer so a single H2D copy refreshes all inputs of a captured step.
// Layout (int64 words):
//   node_s[cs] node_t[ct] eattr_s[es] eattr_t[et] ei_s[2*es] ei_t[2*et]
//   y[cs] ymask[cs] dense_s[cs] dense_t[ct] ptr_s[B+1] ptr_t[B+1]
// Padding: node gather -> zero_node, edge-attr gather -> zero_edge, padded
// edges are self-loops on the padding nodes, dense index -> B*n_max
// (trash slot), y -> 0 with ymask 0.  Returns false (buffer untouched
// semantics irrelevant) if the batch does not fit the capacities.
bool collate_pairs_padded(const Tensor& node_ptr, const Tensor& edge_ptr,
                          const Tensor& edge_local, const Tensor& node_class,
                          const Tensor& pos_of_class, const Tensor& s_ids,
                          const Tensor& t_ids, Tensor out, int64_t cap_s,
                          int64_t cap_t, int64_t ecap_s, int64_t ecap_t,
                          int64_t n_max, int64_t zero_node, int64_t zero_edge,
                          const c10::optional<Tensor>& edge_attr) {
  check_cpu_long(node_ptr, "node_ptr");
  check_cpu_long(edge_ptr, "edge_ptr");
  check_cpu_long(edge_local, "edge_local");
  check_cpu_long(node_class, "node_class");
  check_cpu_long(pos_of_class, "pos_of_class");
  check_cpu_long(s_ids, "s_ids");
  check_cpu_long(t_ids, "t_ids");
  check_cpu_long(out, "out");
  const int64_t B = s_ids.numel();
  TORCH_CHECK(t_ids.numel() == B, "s_ids / t_ids size mismatch");
  // Optional host copy of the edge-attribute table (fp32 [E_all + 1, D]):
  // the attributes are then written into the buffer (no device gather).
  const bool has_ea = edge_attr.has_value() && edge_attr->defined();
  int64_t D = 0;
  if (has_ea) {
    TORCH_CHECK(edge_attr->device().is_cpu() &&
                    edge_attr->scalar_type() == at::kFloat &&
                    edge_attr->dim() == 2 && edge_attr->is_contiguous(),
                "edge_attr must be a contiguous CPU fp32 [E, D] tensor");
    D = edge_attr->size(1);
  }
  const int64_t need = cap_s * 4 + cap_t * 2 + ecap_s * 3 + ecap_t * 3 +
                       2 * (B + 1) + 2 * B + 2 * ecap_t + (cap_s + 7) / 8 +
                       (B + 1) + B + ((ecap_s + ecap_t) * D + 1) / 2;
  // The buffer layout (datasets/static_batch.py::_views) is sized for exactly
  // B pairs: any other count would shift every region after dense_t.
  TORCH_CHECK(out.numel() == need,
              "collate_pairs_padded: buffer size does not match B pairs at "
              "these capacities");
  const int64_t G = node_ptr.numel() - 1;
  const int64_t C = pos_of_class.size(1);
  const int64_t E_all = edge_local.size(1);
  const int64_t* np_ = node_ptr.data_ptr<int64_t>();
  const int64_t* ep_ = edge_ptr.data_ptr<int64_t>();
  const int64_t* src_ = edge_local.data_ptr<int64_t>();
  const int64_t* dst_ = src_ + E_all;
  const int64_t* cls_ = node_class.data_ptr<int64_t>();
  const int64_t* poc_ = pos_of_class.data_ptr<int64_t>();
  const int64_t* sid = s_ids.data_ptr<int64_t>();
  const int64_t* tid = t_ids.data_ptr<int64_t>();

  std::vector<int64_t> ns_off(B + 1, 0), nt_off(B + 1, 0), es_off(B + 1, 0),
      et_off(B + 1, 0);
  for (int64_t b = 0; b < B; ++b) {
    const int64_t gs = sid[b], gt = tid[b];
    TORCH_CHECK(gs >= 0 && gs < G && gt >= 0 && gt < G, "graph id out of range");
    const int64_t cs = np_[gs + 1] - np_[gs], ct = np_[gt + 1] - np_[gt];
    TORCH_CHECK(cs <= n_max && ct <= n_max, "graph larger than n_max");
    ns_off[b + 1] = ns_off[b] + cs;
    nt_off[b + 1] = nt_off[b] + ct;
    es_off[b + 1] = es_off[b] + (ep_[gs + 1] - ep_[gs]);
    et_off[b + 1] = et_off[b] + (ep_[gt + 1] - ep_[gt]);
  }
  // At least one padding node per side hosts the padded edges.
  if (ns_off[B] >= cap_s || nt_off[B] >= cap_t || es_off[B] > ecap_s ||
      et_off[B] > ecap_t)
    return false;

  // Layout (int64 words; see datasets/static_batch.py::_views).  Source and
  // target regions of nodes / edge attributes / edge endpoints are adjacent,
  // so the disjoint union [s; t] psi_1/psi_2 run on is a VIEW of the buffer:
  // target edge endpoints are stored offset by cap_s (union numbering).
  int64_t* o = out.data_ptr<int64_t>();
  int64_t* node_s = o;            o += cap_s;
  int64_t* node_t = o;            o += cap_t;
  int64_t* ea_s = o;              o += ecap_s;
  int64_t* ea_t = o;              o += ecap_t;
  int64_t* ei_s0 = o;             o += ecap_s;
  int64_t* ei_t0 = o;             o += ecap_t;
  int64_t* ei_s1 = o;             o += ecap_s;
  int64_t* ei_t1 = o;             o += ecap_t;
  int64_t* yv = o;                o += cap_s;
  int64_t* ym = o;                o += cap_s;
  int64_t* dn_s = o;              o += cap_s;
  int64_t* dn_t = o;              o += cap_t;
  int64_t* ptr_s = o;             o += B + 1;
  int64_t* ptr_t = o;             o += B + 1;
  int64_t* gid = o;               o += 2 * B;   // store ids: [s_ids; t_ids]
  // Typed tail: the views the step consumes in their final dtype (no cast /
  // subtraction kernels on the device).
  int64_t* ei_tl = o;             o += 2 * ecap_t;  // target edges, local ids
  uint8_t* ymb = reinterpret_cast<uint8_t*>(o);  o += (cap_s + 7) / 8;
  int32_t* p32 = reinterpret_cast<int32_t*>(o);  o += B + 1;  // [ptr_s; ptr_t]
  int32_t* c32 = reinterpret_cast<int32_t*>(o);  o += B;      // [n_s; n_t]
  float* eav = reinterpret_cast<float*>(o);      // [(ecap_s + ecap_t), D]
  const int64_t trash = B * n_max;

#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    const int64_t gs = sid[b], gt = tid[b];
    const int64_t n0s = np_[gs], nns = np_[gs + 1] - n0s;
    const int64_t n0t = np_[gt], nnt = np_[gt + 1] - n0t;
    for (int64_t i = 0; i < nns; ++i) {
      const int64_t r = ns_off[b] + i;
      node_s[r] = n0s + i;
      const int64_t c = cls_[n0s + i];
      const int64_t yy = (c >= 0 && c < C) ? poc_[gt * C + c] : -1;
      yv[r] = yy >= 0 ? yy : 0;
      ym[r] = yy >= 0 ? 1 : 0;
      dn_s[r] = b * n_max + i;
    }
    for (int64_t i = 0; i < nnt; ++i) {
      const int64_t r = nt_off[b] + i;
      node_t[r] = n0t + i;
      dn_t[r] = b * n_max + i;
    }
    const int64_t e0s = ep_[gs], nes = ep_[gs + 1] - e0s;
    for (int64_t e = 0; e < nes; ++e) {
      const int64_t r = es_off[b] + e;
      ea_s[r] = e0s + e;
      ei_s0[r] = src_[e0s + e] + ns_off[b];
      ei_s1[r] = dst_[e0s + e] + ns_off[b];
    }
    const int64_t e0t = ep_[gt], net = ep_[gt + 1] - e0t;
    for (int64_t e = 0; e < net; ++e) {
      const int64_t r = et_off[b] + e;
      ea_t[r] = e0t + e;
      ei_t0[r] = src_[e0t + e] + nt_off[b] + cap_s;
      ei_t1[r] = dst_[e0t + e] + nt_off[b] + cap_s;
    }
  }
  for (int64_t r = ns_off[B]; r < cap_s; ++r) {
    node_s[r] = zero_node; yv[r] = 0; ym[r] = 0; dn_s[r] = trash;
  }
  for (int64_t r = nt_off[B]; r < cap_t; ++r) {
    node_t[r] = zero_node; dn_t[r] = trash;
  }
  // Padded edges are self-loops spread round-robin over ALL padding nodes so
  // no single row of the sparse operators becomes a hub (one hub row of
  // ~1k entries serialised a whole SpMM launch).
  const int64_t pad_s = cap_s - ns_off[B], pad_t = cap_t - nt_off[B];
  for (int64_t r = es_off[B]; r < ecap_s; ++r) {
    const int64_t node = ns_off[B] + (r - es_off[B]) % pad_s;
    ea_s[r] = zero_edge; ei_s0[r] = node; ei_s1[r] = node;
  }
  for (int64_t r = et_off[B]; r < ecap_t; ++r) {
    const int64_t node = nt_off[B] + (r - et_off[B]) % pad_t + cap_s;
    ea_t[r] = zero_edge; ei_t0[r] = node; ei_t1[r] = node;
  }
  for (int64_t b = 0; b <= B; ++b) {
    ptr_s[b] = ns_off[b];
    ptr_t[b] = nt_off[b];
  }
  for (int64_t b = 0; b < B; ++b) {
    gid[b] = sid[b];
    gid[B + b] = tid[b];
  }
  for (int64_t r = 0; r < ecap_t; ++r) {
    ei_tl[r] = ei_t0[r] - cap_s;
    ei_tl[ecap_t + r] = ei_t1[r] - cap_s;
  }
  for (int64_t r = 0; r < cap_s; ++r) ymb[r] = (uint8_t)(ym[r] != 0);
  for (int64_t b = 0; b <= B; ++b) {
    p32[b] = (int32_t)ns_off[b];
    p32[B + 1 + b] = (int32_t)nt_off[b];
  }
  for (int64_t b = 0; b < B; ++b) {
    c32[b] = (int32_t)(ns_off[b + 1] - ns_off[b]);
    c32[B + b] = (int32_t)(nt_off[b + 1] - nt_off[b]);
  }
  if (has_ea) {
    const float* ea = edge_attr->data_ptr<float>();
    const int64_t E_tab = edge_attr->size(0);
    const int64_t ne = ecap_s + ecap_t;
    int64_t bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (int64_t r = 0; r < ne; ++r) {
      const int64_t e = ea_s[r];      // ea_s and ea_t are adjacent
      if (e < 0 || e >= E_tab) {
        ++bad;
        continue;
      }
      for (int64_t d = 0; d < D; ++d) eav[r * D + d] = ea[e * D + d];
    }
    TORCH_CHECK(bad == 0, "collate_pairs_padded: edge id out of range");
  }
  return true;
}

// CSR (rowptr, perm) of an index vector over [0, n): stable counting sort.
std::vector<Tensor> counting_sort(const Tensor& index, int64_t n) {
  check_cpu_long(index, "index");
  const int64_t m = index.numel();
  const int64_t* ix = index.data_ptr<int64_t>();
  Tensor rowptr = at::zeros({n + 1}, at::TensorOptions().dtype(at::kLong));
  Tensor perm = at::empty({m}, at::TensorOptions().dtype(at::kLong));
  int64_t* rp = rowptr.data_ptr<int64_t>();
  for (int64_t i = 0; i < m; ++i) {
    TORCH_CHECK(ix[i] >= 0 && ix[i] < n, "counting_sort: index out of range");
    ++rp[ix[i] + 1];
  }
  for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
  std::vector<int64_t> cursor(rp, rp + n);
  int64_t* pp = perm.data_ptr<int64_t>();
  for (int64_t i = 0; i < m; ++i) pp[cursor[ix[i]]++] = i;
  return {rowptr, perm};
}

}  // namespace dgmc_host

TORCH_LIBRARY(dgmc_host, m) {
  m.def(
      "collate_pairs(Tensor node_ptr, Tensor edge_ptr, Tensor edge_local, "
      "Tensor node_class, Tensor pos_of_class, Tensor s_ids, Tensor t_ids) -> "
      "Tensor[]");
  m.def("counting_sort(Tensor index, int n) -> Tensor[]");
  m.def(
      "collate_pairs_padded(Tensor node_ptr, Tensor edge_ptr, Tensor "
      "edge_local, Tensor node_class, Tensor pos_of_class, Tensor s_ids, "
      "Tensor t_ids, Tensor(a!) out, int cap_s, int cap_t, int ecap_s, int "
      "ecap_t, int n_max, int zero_node, int zero_edge, Tensor? edge_attr=None) "
      "-> bool");
}

TORCH_LIBRARY_IMPL(dgmc_host, CPU, m) {
  m.impl("collate_pairs", &dgmc_host::collate_pairs);
  m.impl("counting_sort", &dgmc_host::counting_sort);
  m.impl("collate_pairs_padded", &dgmc_host::collate_pairs_padded);
}
