// Host sanitizer driver for the native pair collator (csrc/host/collate.cpp).
//
// Built by tools/asan_host.sh with -fsanitize=address,undefined (host code
// only; GPU sanitizers are not available on this pool) and linked against
// libtorch.  Random graph stores and batches exercise every collator entry
// point with buffers allocated at EXACTLY the sizes the kernels assume, so
// any out-of-bounds read/write, use-after-free or UB (signed overflow,
// misaligned access) aborts the run with a sanitizer report.
#include <ATen/ATen.h>

#include <cstdio>
#include <random>
#include <vector>

namespace dgmc_host {
std::vector<at::Tensor> collate_pairs(const at::Tensor& node_ptr,
                                      const at::Tensor& edge_ptr,
                                      const at::Tensor& edge_local,
                                      const at::Tensor& node_class,
                                      const at::Tensor& pos_of_class,
                                      const at::Tensor& s_ids,
                                      const at::Tensor& t_ids);
bool collate_pairs_padded(const at::Tensor& node_ptr,
                          const at::Tensor& edge_ptr,
                          const at::Tensor& edge_local,
                          const at::Tensor& node_class,
                          const at::Tensor& pos_of_class,
                          const at::Tensor& s_ids, const at::Tensor& t_ids,
                          at::Tensor out, int64_t cap_s, int64_t cap_t,
                          int64_t ecap_s, int64_t ecap_t, int64_t n_max,
                          int64_t zero_node, int64_t zero_edge,
                          const c10::optional<at::Tensor>& edge_attr);
std::vector<at::Tensor> counting_sort(const at::Tensor& index, int64_t n);
}  // namespace dgmc_host

#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d %s\n", __FILE__, __LINE__, #cond); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

static at::Tensor longs(const std::vector<int64_t>& v) {
  at::Tensor t = at::empty({(int64_t)v.size()}, at::kLong);
  std::copy(v.begin(), v.end(), t.data_ptr<int64_t>());
  return t;
}

int main() {
  std::mt19937_64 rng(12345);
  auto uni = [&](int64_t lo, int64_t hi) {   // [lo, hi]
    return std::uniform_int_distribution<int64_t>(lo, hi)(rng);
  };
  const int64_t G = 96, C = 20, D = 2;
  std::vector<int64_t> node_ptr{0}, edge_ptr{0}, cls, src, dst;
  std::vector<int64_t> poc(G * C, -1);
  int64_t n_max = 0;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t n = uni(1, C);
    n_max = std::max(n_max, n);
    std::vector<int64_t> perm(C);
    for (int64_t c = 0; c < C; ++c) perm[c] = c;
    std::shuffle(perm.begin(), perm.end(), rng);
    for (int64_t i = 0; i < n; ++i) {
      cls.push_back(perm[i]);
      poc[g * C + perm[i]] = i;
    }
    const int64_t e = uni(0, 4 * n);
    for (int64_t k = 0; k < e; ++k) {
      src.push_back(uni(0, n - 1));
      dst.push_back(uni(0, n - 1));
    }
    node_ptr.push_back(node_ptr.back() + n);
    edge_ptr.push_back(edge_ptr.back() + e);
  }
  const int64_t N_all = node_ptr.back(), E_all = edge_ptr.back();
  at::Tensor np_t = longs(node_ptr), ep_t = longs(edge_ptr);
  at::Tensor el = at::empty({2, E_all}, at::kLong);
  std::copy(src.begin(), src.end(), el.data_ptr<int64_t>());
  std::copy(dst.begin(), dst.end(), el.data_ptr<int64_t>() + E_all);
  at::Tensor cls_t = longs(cls);
  at::Tensor poc_t = longs(poc).view({G, C});
  at::Tensor eattr = at::rand({E_all + 1, D});

  for (int trial = 0; trial < 300; ++trial) {
    const int64_t B = uni(1, 40);
    std::vector<int64_t> s(B), t(B);
    int64_t ns = 0, nt = 0, es = 0, et = 0;
    for (int64_t b = 0; b < B; ++b) {
      s[b] = uni(0, G - 1);
      t[b] = uni(0, G - 1);
      ns += node_ptr[s[b] + 1] - node_ptr[s[b]];
      nt += node_ptr[t[b] + 1] - node_ptr[t[b]];
      es += edge_ptr[s[b] + 1] - edge_ptr[s[b]];
      et += edge_ptr[t[b] + 1] - edge_ptr[t[b]];
    }
    at::Tensor s_t = longs(s), t_t = longs(t);

    // 1. variable-size collation
    auto r = dgmc_host::collate_pairs(np_t, ep_t, el, cls_t, poc_t, s_t, t_t);
    EXPECT(r.size() == 11);
    EXPECT(r[0].numel() == ns && r[1].numel() == nt);
    EXPECT(r[4].size(1) == es && r[5].size(1) == et);
    const int64_t* y = r[10].data_ptr<int64_t>();
    for (int64_t i = 0; i < ns; ++i) EXPECT(y[i] >= -1 && y[i] < C);

    // 2. padded static-batch collation into an exactly sized buffer (with
    //    and without the edge-attribute table), and a batch that overflows
    //    its capacities (must be rejected without touching memory)
    for (int with_ea = 0; with_ea < 2; ++with_ea) {
      const int64_t cap_s = ns + 1 + uni(0, 9), cap_t = nt + 1 + uni(0, 9);
      const int64_t ecap_s = es + uni(0, 17), ecap_t = et + uni(0, 17);
      const int64_t Dw = with_ea ? D : 0;
      const int64_t need = cap_s * 4 + cap_t * 2 + ecap_s * 3 + ecap_t * 3 +
                           2 * (B + 1) + 2 * B + 2 * ecap_t +
                           (cap_s + 7) / 8 + (B + 1) + B +
                           ((ecap_s + ecap_t) * Dw + 1) / 2;
      at::Tensor out = at::empty({need}, at::kLong);
      c10::optional<at::Tensor> ea;
      if (with_ea) ea = eattr;
      const bool ok = dgmc_host::collate_pairs_padded(
          np_t, ep_t, el, cls_t, poc_t, s_t, t_t, out, cap_s, cap_t, ecap_s,
          ecap_t, n_max, N_all, E_all, ea);
      EXPECT(ok);
      if (ns > 1) {
        const int64_t small = ns - 1;   // does not fit: rejected
        const int64_t need2 = small * 4 + cap_t * 2 + ecap_s * 3 +
                              ecap_t * 3 + 2 * (B + 1) + 2 * B + 2 * ecap_t +
                              (small + 7) / 8 + (B + 1) + B +
                              ((ecap_s + ecap_t) * Dw + 1) / 2;
        at::Tensor out2 = at::empty({need2}, at::kLong);
        EXPECT(!dgmc_host::collate_pairs_padded(
            np_t, ep_t, el, cls_t, poc_t, s_t, t_t, out2, small, cap_t,
            ecap_s, ecap_t, n_max, N_all, E_all, ea));
      }
    }

    // 3. stable counting sort
    const int64_t n = uni(1, 64), m = uni(0, 500);
    std::vector<int64_t> idx(m);
    for (auto& v : idx) v = uni(0, n - 1);
    auto cs = dgmc_host::counting_sort(longs(idx), n);
    const int64_t* rp = cs[0].data_ptr<int64_t>();
    const int64_t* pp = cs[1].data_ptr<int64_t>();
    EXPECT(rp[0] == 0 && rp[n] == m);
    for (int64_t k = 0; k < n; ++k)
      for (int64_t q = rp[k]; q < rp[k + 1]; ++q) {
        EXPECT(idx[pp[q]] == k);
        if (q > rp[k]) EXPECT(pp[q] > pp[q - 1]);   // stable
      }
  }
  std::printf("asan_collate: ok (300 random batches, %lld graphs)\n",
              (long long)G);
  return 0;
}
