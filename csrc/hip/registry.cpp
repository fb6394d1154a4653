// Operator schemas + CUDA(=HIP)-key registrations for the gfx950 kernels.
// Loaded from Python with torch.ops.load_library (no pybind module), so the
// ops are visible to the dispatcher, the profiler and hipGraph capture.
#include <ATen/ATen.h>
#include <torch/library.h>

namespace dgmc {
void relconv_fwd(const at::Tensor& ptr, const at::Tensor& col,
                 const at::Tensor& split, const at::Tensor& hub,
                 const at::Tensor& xa, const c10::optional<at::Tensor>& xb,
                 const at::Tensor& w1, const at::Tensor& w2,
                 const at::Tensor& wr, const at::Tensor& bias, bool relu,
                 at::Tensor out, const c10::optional<at::Tensor>& xcopy,
                 const c10::optional<at::Tensor>& feat,
                 const c10::optional<at::Tensor>& fold,
                 const c10::optional<at::Tensor>& pq);
void relconv_bwd(const at::Tensor& ptr, const at::Tensor& col,
                 const at::Tensor& w, const at::Tensor& split,
                 const at::Tensor& hub, const at::Tensor& g,
                 const at::Tensor& xa, const c10::optional<at::Tensor>& xb,
                 const at::Tensor& w1, const at::Tensor& w2,
                 const at::Tensor& wr, const c10::optional<at::Tensor>& dadd,
                 at::Tensor dout, int64_t row0, bool mask, at::Tensor part,
                 bool part_acc);
void rel_proj_bwd(const at::Tensor& dpq, const at::Tensor& feat,
                  const at::Tensor& fold, at::Tensor dfeat, at::Tensor part,
                  bool part_acc);
void rel_fold(at::TensorList parts, at::TensorList outs);
at::Tensor gemm_nt_f32(at::TensorList parts, const at::Tensor& bt,
                       const c10::optional<at::Tensor>& bias, bool relu,
                       const c10::optional<at::Tensor>& out, bool x6,
                       bool accumulate, int64_t sched);
at::Tensor gemm_tn_f32(at::TensorList a_parts, at::TensorList b_parts,
                       const c10::optional<at::Tensor>& out, bool accumulate,
                       bool x6, int64_t splits, int64_t cfg);
std::tuple<at::Tensor, at::Tensor> fold_weights_bwd(const at::Tensor& w1,
                                                    const at::Tensor& wf,
                                                    const at::Tensor& g);
int64_t set_cu_reserve(int64_t n);
at::Tensor cu_hog(const at::Tensor& like, int64_t blocks, double usec);
}  // namespace dgmc

namespace dgmc {

at::Tensor spmm_csr(const at::Tensor& rowptr, const at::Tensor& col,
                    const at::Tensor& val, const at::Tensor& x,
                    const c10::optional<at::Tensor>& self_x,
                    const c10::optional<at::Tensor>& self_scale,
                    const c10::optional<at::Tensor>& bias, bool relu,
                    at::ScalarType out_dtype);
std::vector<at::Tensor> spmm_csr_planes(const at::Tensor& rowptr,
                                        const at::Tensor& col,
                                        const at::Tensor& val,
                                        const at::Tensor& x,
                                        const c10::optional<at::Tensor>& bias,
                                        bool relu);
void spmm_csr_out(const at::Tensor& rowptr, const at::Tensor& col,
                  const at::Tensor& val, const at::Tensor& x,
                  const c10::optional<at::Tensor>& self_x,
                  const c10::optional<at::Tensor>& self_scale,
                  const c10::optional<at::Tensor>& bias, bool relu,
                  at::Tensor out);

std::tuple<at::Tensor, at::Tensor> spline_basis(const at::Tensor& pseudo,
                                                const at::Tensor& kernel_size,
                                                const at::Tensor& is_open,
                                                int64_t degree);

at::Tensor dense_masked_softmax(const at::Tensor& S_hat, const at::Tensor& n_s,
                                const at::Tensor& n_t);
at::Tensor dense_masked_softmax_bwd(const at::Tensor& S, const at::Tensor& G,
                                    const at::Tensor& n_s,
                                    const at::Tensor& n_t);
std::tuple<at::Tensor, at::Tensor> dense_softmax_transport(
    const at::Tensor& S_hat, const at::Tensor& r_s, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, int64_t rows_t, bool joint_out,
    const c10::optional<at::Tensor>& planes);
at::Tensor dense_softmax_transport_bwd(const at::Tensor& S,
                                       const at::Tensor& r_s,
                                       const at::Tensor& g,
                                       const at::Tensor& ptr_s,
                                       const at::Tensor& ptr_t,
                                       const c10::optional<at::Tensor>& addend);
at::Tensor dense_consensus(const at::Tensor& S_hat, const at::Tensor& P,
                           const at::Tensor& Q, const at::Tensor& b1,
                           const at::Tensor& w2, const at::Tensor& b2,
                           const at::Tensor& ptr_s, const at::Tensor& ptr_t);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> dense_consensus_bwd(
    const at::Tensor& G, const at::Tensor& P, const at::Tensor& Q,
    const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, const c10::optional<at::Tensor>& dpq_out,
    const c10::optional<at::Tensor>& part, bool accumulate);

std::vector<at::Tensor> candidate_csc(const at::Tensor& S_idx, int64_t n_t);
at::Tensor train_candidates(const at::Tensor& topk, int64_t n_t, int64_t kr,
                            const at::Tensor& gt_row,
                            const at::Tensor& gt_col);
at::Tensor topk_dot(const at::Tensor& h_s, const at::Tensor& h_t, int64_t k,
                    int64_t mode, const c10::optional<at::Tensor>& warm);
std::vector<at::Tensor> topk_dot_refined_stats(const at::Tensor& h_s,
                                               const at::Tensor& h_t,
                                               int64_t k);

at::Tensor sddmm(const at::Tensor& rowptr, const at::Tensor& col,
                 const at::Tensor& A, const at::Tensor& B);
at::Tensor sparse_consensus_fwd(const at::Tensor& rowptr, const at::Tensor& col,
                                const at::Tensor& S_hat, const at::Tensor& P,
                                const at::Tensor& Q, const at::Tensor& b1,
                                const at::Tensor& w2, const at::Tensor& b2);
std::tuple<at::Tensor, at::Tensor> sparse_consensus_fwd_prob(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& S_hat,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2, const at::Tensor& b2, int64_t k);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor>
sparse_consensus_bwd(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& colptr,
    const at::Tensor& row_of, const at::Tensor& perm, const at::Tensor& G,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2, const c10::optional<at::Tensor>& pptr,
    const c10::optional<at::Tensor>& prow,
    const c10::optional<at::Tensor>& pbeg,
    const c10::optional<at::Tensor>& pend,
    const c10::optional<at::Tensor>& prob,
    const c10::optional<at::Tensor>& gS,
    const c10::optional<at::Tensor>& dpq);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> piece_plan(
    const at::Tensor& rowptr, int64_t nnz, int64_t T);
void spmm_split_out(const at::Tensor& rowptr, const at::Tensor& col,
                    const at::Tensor& val, const at::Tensor& short_rows,
                    const at::Tensor& long_rows, const at::Tensor& x,
                    const c10::optional<at::Tensor>& self_x,
                    const c10::optional<at::Tensor>& self_scale,
                    const c10::optional<at::Tensor>& bias, bool relu,
                    at::Tensor out);
void spmm_pieces_out(const at::Tensor& rowptr, const at::Tensor& col,
                     const at::Tensor& val, const c10::optional<at::Tensor>& perm,
                     const at::Tensor& pptr, const at::Tensor& prow,
                     const at::Tensor& pbeg, const at::Tensor& pend,
                     const at::Tensor& x,
                     const c10::optional<at::Tensor>& self_x,
                     const c10::optional<at::Tensor>& self_scale,
                     const c10::optional<at::Tensor>& bias, bool relu,
                     at::Tensor out);

std::tuple<at::Tensor, at::Tensor> relu_bias_bwd(
    const at::Tensor& grad, const at::Tensor& out, bool relu,
    at::ScalarType g_dtype, const c10::optional<at::Tensor>& dbias,
    bool accumulate, const c10::optional<at::Tensor>& part_out);
at::Tensor col_sum(const at::Tensor& src, const c10::optional<at::Tensor>& dst,
                   bool accumulate, const c10::optional<at::Tensor>& part_out);
void reduce_add_rows(const at::Tensor& src, at::Tensor dst, bool accumulate);
at::Tensor cat_rows(at::TensorList srcs, const c10::optional<at::Tensor>& out);
void assemble_slot_plan(const at::Tensor& st_rowptr, const at::Tensor& st_col,
                        const at::Tensor& st_val, const at::Tensor& st_trowptr,
                        const at::Tensor& st_tcol, const at::Tensor& st_tval,
                        const at::Tensor& node_ptr, const at::Tensor& gid,
                        const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                        int64_t cap_s, int64_t cap_t, int64_t S,
                        int64_t root_slot, at::Tensor rowptr, at::Tensor col,
                        at::Tensor val, at::Tensor trowptr, at::Tensor tcol,
                        at::Tensor tval,
                        const c10::optional<at::Tensor>& gflag,
                        const c10::optional<at::Tensor>& st_row,
                        const c10::optional<at::Tensor>& row_out);
at::Tensor masked_softmax_packed(const at::Tensor& S_hat,
                                 const at::Tensor& dense_index,
                                 const at::Tensor& n_s, const at::Tensor& n_t);
at::Tensor masked_softmax_packed_bwd(const at::Tensor& S, const at::Tensor& G,
                                     const at::Tensor& dense_index, int64_t B,
                                     int64_t Ns);
std::tuple<at::Tensor, at::Tensor> nll_fwd(const at::Tensor& S,
                                           const at::Tensor& y0,
                                           const at::Tensor& y1,
                                           const c10::optional<at::Tensor>& mask,
                                           double eps, bool mean,
                                           bool with_correct);
at::Tensor nll_bwd(const at::Tensor& grad, const at::Tensor& S,
                   const at::Tensor& y0, const at::Tensor& y1,
                   const c10::optional<at::Tensor>& mask, const at::Tensor& aux,
                   double eps, bool mean);
std::tuple<at::Tensor, at::Tensor> sparse_nll_fwd(
    const at::Tensor& val, const at::Tensor& idx, const at::Tensor& y0,
    const at::Tensor& y1, const c10::optional<at::Tensor>& mask, double eps,
    bool mean);
at::Tensor sparse_nll_bwd(const at::Tensor& grad, const at::Tensor& val,
                          const at::Tensor& idx, const at::Tensor& y0,
                          const at::Tensor& y1,
                          const c10::optional<at::Tensor>& mask,
                          const at::Tensor& aux, double eps, bool mean);
void nonfinite_flag(const at::Tensor& x, at::Tensor found_inf,
                    const c10::optional<at::Tensor>& counter);
at::Tensor slot_conv_stamps();
std::tuple<at::Tensor, at::Tensor, at::Tensor> fold_weights(
    const at::Tensor& w1, const at::Tensor& wf);
at::Tensor dense_wgrad(at::TensorList xs, at::TensorList gs, int64_t nsplit);
at::Tensor tr16_probe(const at::Tensor& like);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> slot_pair_lists(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& val,
    const at::Tensor& row, int64_t S);
at::Tensor slot_wgrad(const at::Tensor& X, const at::Tensor& G,
                      const at::Tensor& esrc, const at::Tensor& edst,
                      const at::Tensor& evals, const at::Tensor& soff,
                      int64_t U, int64_t nsplit);
void adam_multi(at::TensorList params, at::TensorList grads,
                at::TensorList exp_avg, at::TensorList exp_avg_sq,
                at::TensorList steps,
                const c10::optional<at::Tensor>& found_inf, double lr,
                double beta1, double beta2, double eps, double weight_decay);
void adam_step_inc(at::TensorList steps,
                   const c10::optional<at::Tensor>& found_inf,
                   const c10::optional<at::Tensor>& flags,
                   const c10::optional<at::Tensor>& skips);
at::Tensor slot_wgrad_list(at::TensorList xs, at::TensorList gs,
                           const at::Tensor& esrc, const at::Tensor& edst,
                           const at::Tensor& evals, const at::Tensor& soff,
                           int64_t nsplit);
at::Tensor slot_conv(const at::Tensor& X, const at::Tensor& tiles,
                     const at::Tensor& soff, const at::Tensor& ecode,
                     const at::Tensor& eval, int64_t S, const at::Tensor& Wimg,
                     bool trans, const c10::optional<at::Tensor>& bias,
                     bool relu, at::ScalarType out_dtype,
                     const c10::optional<at::Tensor>& Z,
                     const c10::optional<at::Tensor>& addend);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> slot_tile_plan(
    const at::Tensor& flag, const at::Tensor& rowptr, const at::Tensor& col,
    const at::Tensor& val, int64_t window, int64_t S, at::Tensor err);
at::Tensor gemm_abt(const at::Tensor& A, const at::Tensor& Bt,
                    const c10::optional<at::Tensor>& out, bool accumulate,
                    c10::optional<at::ScalarType> out_dtype);
at::Tensor spline_weight_pack(const at::Tensor& weight,
                              const c10::optional<at::Tensor>& root,
                              at::ScalarType dtype);
std::tuple<at::Tensor, at::Tensor> spline_weight_unpack(const at::Tensor& g,
                                                        int64_t K,
                                                        bool has_root);
at::Tensor pack_grads(const c10::List<c10::optional<at::Tensor>>& grads,
                      at::TensorList views, bool with_flags);
at::Tensor cat_gemm(at::TensorList xs, const at::Tensor& W,
                    const c10::optional<at::Tensor>& ocat);
std::tuple<at::Tensor, at::Tensor, at::Tensor> dense_consensus_transport(
    const at::Tensor& S_hat, const at::Tensor& P, const at::Tensor& Q,
    const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2,
    const at::Tensor& r_s, const at::Tensor& ptr_s, const at::Tensor& ptr_t,
    int64_t rows_t, const c10::optional<at::Tensor>& planes);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
dense_transport_consensus_bwd(const at::Tensor& S_prob, const at::Tensor& r_s,
                              const at::Tensor& g_t,
                              const c10::optional<at::Tensor>& addend,
                              const at::Tensor& P, const at::Tensor& Q,
                              const at::Tensor& b1, const at::Tensor& w2,
                              const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                              const c10::optional<at::Tensor>& dpq_out,
                              const c10::optional<at::Tensor>& part,
                              bool accumulate);
std::tuple<at::Tensor, at::Tensor> softmax_nll_fwd(
    const at::Tensor& S_hat, const c10::optional<at::Tensor>& S_hat2,
    const at::Tensor& ptr_s, const at::Tensor& n_t, const at::Tensor& y,
    const c10::optional<at::Tensor>& mask, double eps,
    const c10::optional<at::Tensor>& stats);
std::tuple<at::Tensor, at::Tensor> softmax_nll_bwd(
    const at::Tensor& grad, const at::Tensor& S_hat,
    const c10::optional<at::Tensor>& S_hat2, const at::Tensor& ptr_s,
    const at::Tensor& n_t, const at::Tensor& y,
    const c10::optional<at::Tensor>& mask, const at::Tensor& aux,
    double eps);
at::Tensor pair_scores(const at::Tensor& h, int64_t t_off,
                       const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                       int64_t Ns, int64_t Nt);
at::Tensor pair_scores_bwd(const at::Tensor& dS, const at::Tensor& h,
                           int64_t t_off, const at::Tensor& ptr_s,
                           const at::Tensor& ptr_t,
                           const c10::optional<at::Tensor>& dS2);
std::tuple<at::Tensor, at::Tensor> spline_slot_images(
    const at::Tensor& weight, const c10::optional<at::Tensor>& root,
    const at::Tensor& perm);
at::Tensor slot_conv_relu_bwd(const at::Tensor& G,
                              const c10::optional<at::Tensor>& relu_out,
                              const at::Tensor& tiles, const at::Tensor& soff,
                              const at::Tensor& ecode, const at::Tensor& eval,
                              int64_t S, const at::Tensor& Wimg,
                              at::ScalarType out_dtype,
                              const c10::optional<at::Tensor>& addend,
                              at::Tensor g_out,
                              const c10::optional<at::Tensor>& bias_part);

std::vector<at::Tensor> slot_compact_plan(const at::Tensor& rowptr,
                                          const at::Tensor& col, int64_t Nsrc,
                                          int64_t S, int64_t P_cap);
at::Tensor slot_gemm(const at::Tensor& X, const at::Tensor& src,
                     const at::Tensor& seg, const at::Tensor& weight,
                     const c10::optional<at::Tensor>& root, bool trans_w,
                     const c10::optional<at::Tensor>& tiles);
at::Tensor slot_dx_tiles(const at::Tensor& src, const at::Tensor& seg,
                         int64_t N, int64_t row0, int64_t P_cap,
                         int64_t unit);
at::Tensor slot_gemm2(const at::Tensor& X, const at::Tensor& src,
                      const at::Tensor& seg, const at::Tensor& bt,
                      const c10::optional<at::Tensor>& broot, bool gather);
at::Tensor split3(const at::Tensor& x);
at::Tensor slot_weight_x3(const at::Tensor& weight,
                          const c10::optional<at::Tensor>& root,
                          bool transpose);
at::Tensor slot_gemm_x6(const at::Tensor& a3, const at::Tensor& src,
                        const at::Tensor& seg, const at::Tensor& b3,
                        bool gather, const c10::optional<at::Tensor>& tiles);
at::Tensor slot_wgrad_x6(at::TensorList xs, at::TensorList gs,
                         const at::Tensor& src, const at::Tensor& seg,
                         int64_t rounds, const c10::optional<at::Tensor>& ell,
                         const c10::optional<at::Tensor>& ecol,
                         const c10::optional<at::Tensor>& evl);
at::Tensor slot_weight_t(const at::Tensor& weight,
                         const c10::optional<at::Tensor>& root);
at::Tensor dense_nt_f32(at::TensorList parts, const at::Tensor& bt);
at::Tensor dense_nt_x6(at::TensorList parts, const at::Tensor& bt,
                       const c10::optional<at::Tensor>& b3);
at::Tensor dense_wgrad_f32(at::TensorList xparts, int64_t nparts,
                           at::TensorList gs, const at::Tensor& seg01);
at::Tensor slot_spmm_rowmap(const at::Tensor& rowptr, const at::Tensor& col,
                            const at::Tensor& val, const at::Tensor& cinv,
                            const at::Tensor& g,
                            const c10::optional<at::Tensor>& seg,
                            const c10::optional<at::Tensor>& ranges,
                            bool planes);
at::Tensor slot_rowmap_ell(const at::Tensor& rowptr, const at::Tensor& col,
                           const at::Tensor& val, const at::Tensor& cinv);
at::Tensor slot_rowmap_ranges(const at::Tensor& rowptr,
                              const at::Tensor& cinv);
at::Tensor slot_gather_sum(const at::Tensor& posmap, const at::Tensor& Z,
                           int64_t N, int64_t S,
                           const c10::optional<at::Tensor>& add,
                           int64_t row0,
                           const c10::optional<at::Tensor>& relu_out,
                           const c10::optional<at::Tensor>& part);
at::Tensor slot_wgrad_f32(at::TensorList xs, at::TensorList gs,
                          const at::Tensor& src, const at::Tensor& seg,
                          int64_t rounds);
std::vector<at::Tensor> sinkhorn_transport(const at::Tensor& S_hat,
                                           const at::Tensor& r_s,
                                           const at::Tensor& ptr_s,
                                           const at::Tensor& ptr_t,
                                           int64_t rows_t, int64_t iters,
                                           double tau, bool with_prob);
at::Tensor sinkhorn_transport_bwd(const c10::optional<at::Tensor>& G,
                                  const at::Tensor& g_joint,
                                  const at::Tensor& r_s,
                                  const at::Tensor& S_hat,
                                  const at::Tensor& ptr_s,
                                  const at::Tensor& ptr_t,
                                  const at::Tensor& a_hist,
                                  const at::Tensor& b_hist, int64_t iters,
                                  double tau,
                                  const c10::optional<at::Tensor>& add);
std::tuple<at::Tensor, at::Tensor, at::Tensor> sinkhorn_fwd(
    const at::Tensor& S_hat, const at::Tensor& n_s, const at::Tensor& n_t,
    int64_t iters, double tau);
at::Tensor sinkhorn_bwd(const at::Tensor& G, const at::Tensor& S_hat,
                        const at::Tensor& n_s, const at::Tensor& n_t,
                        const at::Tensor& a_hist, const at::Tensor& b_hist,
                        int64_t iters, double tau);

}  // namespace dgmc

TORCH_LIBRARY(dgmc_amd, m) {
  m.def("set_cu_reserve(int n) -> int");
  m.def(
      "relconv_fwd(Tensor ptr, Tensor col, Tensor split, Tensor hub, Tensor "
      "xa, Tensor? xb, Tensor w1, Tensor w2, Tensor wr, Tensor bias, bool "
      "relu, Tensor(a!) out, Tensor(b!)? xcopy, Tensor? feat, Tensor? fold, "
      "Tensor(c!)? pq) -> ()");
  m.def(
      "relconv_bwd(Tensor ptr, Tensor col, Tensor w, Tensor split, Tensor "
      "hub, Tensor g, Tensor xa, Tensor? xb, Tensor w1, Tensor w2, Tensor wr, "
      "Tensor? dadd, Tensor(a!) dout, int row0, bool mask, Tensor(b!) part, "
      "bool part_acc) -> ()");
  m.def("rel_fold(Tensor[] parts, Tensor(a!)[] outs) -> ()");
  m.def(
      "gemm_nt_f32(Tensor[] parts, Tensor bt, Tensor? bias=None, bool "
      "relu=False, Tensor(a!)? out=None, bool x6=False, bool accumulate="
      "False, int sched=0) -> Tensor");
  m.def(
      "gemm_tn_f32(Tensor[] a_parts, Tensor[] b_parts, Tensor(a!)? out=None, "
      "bool accumulate=False, bool x6=True, int splits=0, int cfg=0) -> "
      "Tensor");
  m.def("fold_weights_bwd(Tensor w1, Tensor wf, Tensor g) -> (Tensor, Tensor)");
  m.def(
      "rel_proj_bwd(Tensor dpq, Tensor feat, Tensor fold, Tensor(a!) dfeat, "
      "Tensor(b!) part, bool part_acc) -> ()");
  m.def("cu_hog(Tensor like, int blocks, float usec) -> Tensor");
  m.def(
      "spmm_csr(Tensor rowptr, Tensor col, Tensor val, Tensor x, Tensor? "
      "self_x, Tensor? self_scale, Tensor? bias, bool relu, ScalarType "
      "out_dtype) -> "
      "Tensor");
  m.def(
      "spmm_csr_planes(Tensor rowptr, Tensor col, Tensor val, Tensor x, "
      "Tensor? bias, bool relu) -> Tensor[]");
  m.def(
      "spmm_csr_out(Tensor rowptr, Tensor col, Tensor val, Tensor x, Tensor? "
      "self_x, Tensor? self_scale, Tensor? bias, bool relu, Tensor(a!) out) "
      "-> ()");
  m.def(
      "spline_basis(Tensor pseudo, Tensor kernel_size, Tensor is_open, int "
      "degree) -> (Tensor, Tensor)");
  m.def("dense_masked_softmax(Tensor S_hat, Tensor n_s, Tensor n_t) -> Tensor");
  m.def(
      "dense_masked_softmax_bwd(Tensor S, Tensor grad, Tensor n_s, Tensor n_t) "
      "-> Tensor");
  m.def(
      "dense_softmax_transport(Tensor S_hat, Tensor r_s, Tensor ptr_s, Tensor "
      "ptr_t, int rows_t, bool joint_out=False, Tensor(a!)? planes=None) -> "
      "(Tensor, Tensor)");
  m.def(
      "dense_softmax_transport_bwd(Tensor S, Tensor r_s, Tensor grad, Tensor "
      "ptr_s, Tensor ptr_t, Tensor? addend=None) -> Tensor");
  m.def(
      "dense_consensus(Tensor S_hat, Tensor P, Tensor Q, Tensor b1, Tensor w2, "
      "Tensor b2, Tensor ptr_s, Tensor ptr_t) -> Tensor");
  m.def(
      "dense_consensus_bwd(Tensor grad, Tensor P, Tensor Q, Tensor b1, Tensor "
      "w2, Tensor ptr_s, Tensor ptr_t, Tensor(a!)? dpq_out=None, Tensor(b!)? "
      "part=None, bool accumulate=False) -> (Tensor, Tensor, Tensor, "
      "Tensor)");
  m.def(
      "topk_dot(Tensor h_s, Tensor h_t, int k, int mode=2, Tensor(a!)? "
      "warm=None) -> Tensor");
  m.def("topk_dot_refined_stats(Tensor h_s, Tensor h_t, int k) -> Tensor[]");
  m.def("train_candidates(Tensor topk, int n_t, int kr, Tensor gt_row, "
        "Tensor gt_col) -> Tensor");
  m.def("candidate_csc(Tensor S_idx, int n_t) -> Tensor[]");
  m.def("sddmm(Tensor rowptr, Tensor col, Tensor A, Tensor B) -> Tensor");
  m.def(
      "relu_bias_bwd(Tensor grad, Tensor out, bool relu, ScalarType g_dtype, "
      "Tensor(a!)? dbias=None, bool accumulate=False, Tensor(b!)? "
      "part_out=None) -> (Tensor, Tensor)");
  m.def(
      "col_sum(Tensor src, Tensor(a!)? dst=None, bool accumulate=False, "
      "Tensor(b!)? part_out=None) -> Tensor");
  m.def("reduce_add_rows(Tensor src, Tensor(a!) dst, bool accumulate) -> ()");
  m.def("cat_rows(Tensor[] srcs, Tensor(a!)? out=None) -> Tensor");
  m.def(
      "masked_softmax_packed(Tensor S_hat, Tensor dense_index, Tensor n_s, "
      "Tensor n_t) -> Tensor");
  m.def(
      "masked_softmax_packed_bwd(Tensor S, Tensor grad, Tensor dense_index, "
      "int B, int Ns) -> Tensor");
  m.def(
      "nll_fwd(Tensor S, Tensor y0, Tensor y1, Tensor? mask, float eps, bool "
      "mean, bool with_correct) -> (Tensor, Tensor)");
  m.def(
      "nll_bwd(Tensor grad, Tensor S, Tensor y0, Tensor y1, Tensor? mask, "
      "Tensor aux, float eps, bool mean) -> Tensor");
  m.def(
      "sparse_nll_fwd(Tensor val, Tensor idx, Tensor y0, Tensor y1, Tensor? "
      "mask, float eps, bool mean) -> (Tensor, Tensor)");
  m.def(
      "sparse_nll_bwd(Tensor grad, Tensor val, Tensor idx, Tensor y0, Tensor "
      "y1, Tensor? mask, Tensor aux, float eps, bool mean) -> Tensor");
  m.def(
      "nonfinite_flag(Tensor x, Tensor(a!) found_inf, Tensor(b!)? counter=None)"
      " -> ()");
  m.def(
      "assemble_slot_plan(Tensor st_rowptr, Tensor st_col, Tensor st_val, "
      "Tensor st_trowptr, Tensor st_tcol, Tensor st_tval, Tensor node_ptr, "
      "Tensor gid, Tensor ptr_s, Tensor ptr_t, int cap_s, int cap_t, int S, "
      "int root_slot, Tensor(a!) rowptr, Tensor(b!) col, Tensor(c!) val, "
      "Tensor(d!) trowptr, Tensor(e!) tcol, Tensor(f!) tval, Tensor(g!)? "
      "gflag=None, Tensor? st_row=None, Tensor(h!)? row_out=None) -> ()");
  m.def("slot_conv_stamps() -> Tensor");
  m.def("fold_weights(Tensor w1, Tensor wf) -> (Tensor, Tensor, Tensor)");
  m.def("dense_wgrad(Tensor[] xs, Tensor[] gs, int nsplit) -> Tensor");
  m.def("tr16_probe(Tensor like) -> Tensor");
  m.def(
      "slot_pair_lists(Tensor rowptr, Tensor col, Tensor val, Tensor row, int "
      "S) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "slot_wgrad(Tensor X, Tensor G, Tensor esrc, Tensor edst, Tensor evals, "
      "Tensor soff, int U, int nsplit) -> Tensor");
  m.def(
      "adam_multi(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avg, "
      "Tensor(c!)[] exp_avg_sq, Tensor[] steps, Tensor? found_inf, float lr, "
      "float beta1, float beta2, float eps, float weight_decay) -> ()");
  m.def(
      "adam_step_inc(Tensor(a!)[] steps, Tensor(b!)? found_inf, "
      "Tensor? flags=None, Tensor(c!)? skips=None) -> ()");
  m.def(
      "spline_weight_pack(Tensor weight, Tensor? root, ScalarType dtype) -> "
      "Tensor");
  m.def(
      "spline_weight_unpack(Tensor g, int K, bool has_root) -> (Tensor, "
      "Tensor)");
  m.def("pack_grads(Tensor?[] grads, Tensor(a!)[] views, bool with_flags=False) -> Tensor");
  m.def("cat_gemm(Tensor[] xs, Tensor W, Tensor(a!)? ocat=None) -> Tensor");
  m.def(
      "dense_consensus_transport(Tensor S_hat, Tensor P, Tensor Q, Tensor b1, "
      "Tensor w2, Tensor b2, Tensor r_s, Tensor ptr_s, Tensor ptr_t, int "
      "rows_t, Tensor(a!)? planes=None) -> (Tensor, Tensor, Tensor)");
  m.def(
      "dense_transport_consensus_bwd(Tensor S, Tensor r_s, Tensor g_t, "
      "Tensor? addend, Tensor P, Tensor Q, Tensor b1, Tensor w2, Tensor "
      "ptr_s, Tensor ptr_t, Tensor(a!)? dpq_out=None, Tensor(b!)? part=None, "
      "bool accumulate=False) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "softmax_nll_fwd(Tensor S_hat, Tensor? S_hat2, Tensor ptr_s, Tensor "
      "n_t, Tensor y, Tensor? mask, float eps, Tensor(a!)? stats=None) -> "
      "(Tensor, Tensor)");
  m.def(
      "softmax_nll_bwd(Tensor grad, Tensor S_hat, Tensor? S_hat2, Tensor "
      "ptr_s, Tensor n_t, Tensor y, Tensor? mask, Tensor aux, float eps) -> "
      "(Tensor, Tensor)");
  m.def(
      "pair_scores(Tensor h, int t_off, Tensor ptr_s, Tensor ptr_t, int Ns, "
      "int Nt) -> Tensor");
  m.def(
      "pair_scores_bwd(Tensor dS, Tensor h, int t_off, Tensor ptr_s, Tensor "
      "ptr_t, Tensor? dS2=None) -> Tensor");
  m.def(
      "spline_slot_images(Tensor weight, Tensor? root, Tensor perm) -> "
      "(Tensor, Tensor)");
  m.def(
      "slot_conv_relu_bwd(Tensor G, Tensor? relu_out, Tensor tiles, Tensor "
      "soff, Tensor ecode, Tensor eval, int S, Tensor Wimg, ScalarType "
      "out_dtype, Tensor? addend, Tensor(a!) g_out, Tensor(b!)? bias_part) -> "
      "Tensor");
  m.def(
      "slot_wgrad_list(Tensor[] xs, Tensor[] gs, Tensor esrc, Tensor edst, "
      "Tensor evals, Tensor soff, int nsplit) -> Tensor");
  m.def(
      "slot_conv(Tensor X, Tensor tiles, Tensor soff, Tensor ecode, Tensor "
      "eval, int S, Tensor Wimg, bool trans, Tensor? bias, bool relu, "
      "ScalarType out_dtype, Tensor(a!)? Z=None, Tensor? addend=None) -> "
      "Tensor");
  m.def(
      "slot_tile_plan(Tensor flag, Tensor rowptr, Tensor col, Tensor val, int "
      "window, int S, Tensor(a!) err) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "gemm_abt(Tensor A, Tensor Bt, Tensor(a!)? out=None, bool "
      "accumulate=False, ScalarType? out_dtype=None) -> Tensor");
  m.def(
      "sparse_consensus_fwd(Tensor rowptr, Tensor col, Tensor S_hat, Tensor P, "
      "Tensor Q, Tensor b1, Tensor w2, Tensor b2) -> Tensor");
  m.def(
      "sparse_consensus_bwd(Tensor rowptr, Tensor col, Tensor colptr, Tensor "
      "row_of, Tensor perm, Tensor grad, Tensor P, Tensor Q, Tensor b1, Tensor "
      "w2, Tensor? pptr=None, Tensor? prow=None, Tensor? pbeg=None, Tensor? "
      "pend=None, Tensor? prob=None, Tensor? gS=None, Tensor(a!)? dpq=None) "
      "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "sparse_consensus_fwd_prob(Tensor rowptr, Tensor col, Tensor S_hat, "
      "Tensor P, Tensor Q, Tensor b1, Tensor w2, Tensor b2, int k) -> (Tensor, "
      "Tensor)");
  m.def(
      "piece_plan(Tensor rowptr, int nnz, int T) -> (Tensor, Tensor, Tensor, "
      "Tensor)");
  m.def(
      "spmm_pieces_out(Tensor rowptr, Tensor col, Tensor val, Tensor? perm, "
      "Tensor pptr, Tensor prow, Tensor pbeg, Tensor pend, Tensor x, Tensor? "
      "self_x, Tensor? self_scale, Tensor? bias, bool relu, Tensor(a!) out) -> "
      "()");
  m.def(
      "spmm_split_out(Tensor rowptr, Tensor col, Tensor val, Tensor short_rows, "
      "Tensor long_rows, Tensor x, Tensor? self_x, Tensor? self_scale, "
      "Tensor? bias, bool relu, Tensor(a!) out) -> ()");
  m.def(
      "slot_compact_plan(Tensor rowptr, Tensor col, int Nsrc, int S, int "
      "P_cap) -> Tensor[]");
  m.def(
      "slot_gemm(Tensor X, Tensor src, Tensor seg, Tensor weight, Tensor? "
      "root, bool trans_w, Tensor? tiles=None) -> Tensor");
  m.def(
      "slot_dx_tiles(Tensor src, Tensor seg, int N, int row0, int P_cap, "
      "int unit=128) -> Tensor");
  m.def(
      "slot_gemm2(Tensor X, Tensor src, Tensor seg, Tensor bt, Tensor? "
      "broot, bool gather) -> Tensor");
  m.def("slot_weight_t(Tensor weight, Tensor? root) -> Tensor");
  m.def("split3(Tensor x) -> Tensor");
  m.def(
      "slot_wgrad_x6(Tensor[] xs, Tensor[] gs, Tensor src, Tensor seg, int "
      "rounds, Tensor? ell=None, Tensor? ecol=None, Tensor? evl=None) -> "
      "Tensor");
  m.def("slot_weight_x3(Tensor weight, Tensor? root, bool transpose) -> Tensor");
  m.def(
      "slot_gemm_x6(Tensor a3, Tensor src, Tensor seg, Tensor b3, bool gather, "
      "Tensor? tiles=None) -> Tensor");
  m.def("dense_nt_f32(Tensor[] parts, Tensor bt) -> Tensor");
  m.def("dense_nt_x6(Tensor[] parts, Tensor bt, Tensor? b3=None) -> Tensor");
  m.def(
      "dense_wgrad_f32(Tensor[] xparts, int nparts, Tensor[] gs, Tensor "
      "seg01) -> Tensor");
  m.def(
      "slot_spmm_rowmap(Tensor rowptr, Tensor col, Tensor val, Tensor cinv, "
      "Tensor g, Tensor? seg=None, Tensor? ranges=None, bool planes=False) -> "
      "Tensor");
  m.def("slot_rowmap_ranges(Tensor rowptr, Tensor cinv) -> Tensor");
  m.def("slot_rowmap_ell(Tensor rowptr, Tensor col, Tensor val, Tensor cinv) "
        "-> Tensor");
  m.def(
      "slot_gather_sum(Tensor posmap, Tensor Z, int N, int S, Tensor? add, "
      "int row0=0, Tensor? relu_out=None, Tensor(a!)? part=None) -> Tensor");
  m.def(
      "slot_wgrad_f32(Tensor[] xs, Tensor[] gs, Tensor src, Tensor seg, int "
      "rounds) -> Tensor");
  m.def(
      "sinkhorn_fwd(Tensor S_hat, Tensor n_s, Tensor n_t, int iters, float "
      "tau) -> (Tensor, Tensor, Tensor)");
  m.def(
      "sinkhorn_bwd(Tensor grad, Tensor S_hat, Tensor n_s, Tensor n_t, Tensor "
      "a_hist, Tensor b_hist, int iters, float tau) -> Tensor");
  m.def(
      "sinkhorn_transport(Tensor S_hat, Tensor r_s, Tensor ptr_s, Tensor "
      "ptr_t, int rows_t, int iters, float tau, bool with_prob) -> Tensor[]");
  m.def(
      "sinkhorn_transport_bwd(Tensor? grad_P, Tensor grad_joint, Tensor r_s, "
      "Tensor S_hat, Tensor ptr_s, Tensor ptr_t, Tensor a_hist, Tensor "
      "b_hist, int iters, float tau, Tensor? add) -> Tensor");
}

TORCH_LIBRARY_IMPL(dgmc_amd, CompositeExplicitAutograd, m) {
  m.impl("slot_conv_stamps", &dgmc::slot_conv_stamps);
  m.impl("set_cu_reserve", &dgmc::set_cu_reserve);
}

TORCH_LIBRARY_IMPL(dgmc_amd, CUDA, m) {
  m.impl("cu_hog", &dgmc::cu_hog);
  m.impl("relconv_fwd", &dgmc::relconv_fwd);
  m.impl("relconv_bwd", &dgmc::relconv_bwd);
  m.impl("rel_proj_bwd", &dgmc::rel_proj_bwd);
  m.impl("fold_weights_bwd", &dgmc::fold_weights_bwd);
  m.impl("rel_fold", &dgmc::rel_fold);
  m.impl("gemm_nt_f32", &dgmc::gemm_nt_f32);
  m.impl("gemm_tn_f32", &dgmc::gemm_tn_f32);
  m.impl("spmm_csr", &dgmc::spmm_csr);
  m.impl("spmm_csr_planes", &dgmc::spmm_csr_planes);
  m.impl("spmm_csr_out", &dgmc::spmm_csr_out);
  m.impl("spline_basis", &dgmc::spline_basis);
  m.impl("dense_masked_softmax", &dgmc::dense_masked_softmax);
  m.impl("dense_masked_softmax_bwd", &dgmc::dense_masked_softmax_bwd);
  m.impl("dense_softmax_transport", &dgmc::dense_softmax_transport);
  m.impl("dense_softmax_transport_bwd", &dgmc::dense_softmax_transport_bwd);
  m.impl("dense_consensus", &dgmc::dense_consensus);
  m.impl("dense_consensus_bwd", &dgmc::dense_consensus_bwd);
  m.impl("topk_dot", &dgmc::topk_dot);
  m.impl("topk_dot_refined_stats", &dgmc::topk_dot_refined_stats);
  m.impl("train_candidates", &dgmc::train_candidates);
  m.impl("candidate_csc", &dgmc::candidate_csc);
  m.impl("sddmm", &dgmc::sddmm);
  m.impl("relu_bias_bwd", &dgmc::relu_bias_bwd);
  m.impl("col_sum", &dgmc::col_sum);
  m.impl("reduce_add_rows", &dgmc::reduce_add_rows);
  m.impl("cat_rows", &dgmc::cat_rows);
  m.impl("masked_softmax_packed", &dgmc::masked_softmax_packed);
  m.impl("masked_softmax_packed_bwd", &dgmc::masked_softmax_packed_bwd);
  m.impl("nll_fwd", &dgmc::nll_fwd);
  m.impl("nll_bwd", &dgmc::nll_bwd);
  m.impl("sparse_nll_fwd", &dgmc::sparse_nll_fwd);
  m.impl("sparse_nll_bwd", &dgmc::sparse_nll_bwd);
  m.impl("nonfinite_flag", &dgmc::nonfinite_flag);
  m.impl("assemble_slot_plan", &dgmc::assemble_slot_plan);
  m.impl("slot_conv", &dgmc::slot_conv);
  m.impl("slot_tile_plan", &dgmc::slot_tile_plan);
  m.impl("slot_wgrad", &dgmc::slot_wgrad);
  m.impl("slot_wgrad_list", &dgmc::slot_wgrad_list);
  m.impl("adam_multi", &dgmc::adam_multi);
  m.impl("adam_step_inc", &dgmc::adam_step_inc);
  m.impl("spline_weight_pack", &dgmc::spline_weight_pack);
  m.impl("spline_weight_unpack", &dgmc::spline_weight_unpack);
  m.impl("slot_conv_relu_bwd", &dgmc::slot_conv_relu_bwd);
  m.impl("pack_grads", &dgmc::pack_grads);
  m.impl("cat_gemm", &dgmc::cat_gemm);
  m.impl("dense_consensus_transport", &dgmc::dense_consensus_transport);
  m.impl("dense_transport_consensus_bwd",
         &dgmc::dense_transport_consensus_bwd);
  m.impl("softmax_nll_fwd", &dgmc::softmax_nll_fwd);
  m.impl("softmax_nll_bwd", &dgmc::softmax_nll_bwd);
  m.impl("pair_scores", &dgmc::pair_scores);
  m.impl("pair_scores_bwd", &dgmc::pair_scores_bwd);
  m.impl("spline_slot_images", &dgmc::spline_slot_images);
  m.impl("tr16_probe", &dgmc::tr16_probe);
  m.impl("dense_wgrad", &dgmc::dense_wgrad);
  m.impl("fold_weights", &dgmc::fold_weights);
  m.impl("slot_pair_lists", &dgmc::slot_pair_lists);
  m.impl("gemm_abt", &dgmc::gemm_abt);
  m.impl("sparse_consensus_fwd", &dgmc::sparse_consensus_fwd);
  m.impl("sparse_consensus_bwd", &dgmc::sparse_consensus_bwd);
  m.impl("sparse_consensus_fwd_prob", &dgmc::sparse_consensus_fwd_prob);
  m.impl("spmm_pieces_out", &dgmc::spmm_pieces_out);
  m.impl("spmm_split_out", &dgmc::spmm_split_out);
  m.impl("piece_plan", &dgmc::piece_plan);
  m.impl("slot_compact_plan", &dgmc::slot_compact_plan);
  m.impl("slot_gemm", &dgmc::slot_gemm);
  m.impl("slot_gemm2", &dgmc::slot_gemm2);
  m.impl("slot_dx_tiles", &dgmc::slot_dx_tiles);
  m.impl("slot_weight_t", &dgmc::slot_weight_t);
  m.impl("split3", &dgmc::split3);
  m.impl("slot_wgrad_x6", &dgmc::slot_wgrad_x6);
  m.impl("slot_weight_x3", &dgmc::slot_weight_x3);
  m.impl("slot_gemm_x6", &dgmc::slot_gemm_x6);
  m.impl("dense_nt_f32", &dgmc::dense_nt_f32);
  m.impl("dense_nt_x6", &dgmc::dense_nt_x6);
  m.impl("dense_wgrad_f32", &dgmc::dense_wgrad_f32);
  m.impl("slot_spmm_rowmap", &dgmc::slot_spmm_rowmap);
  m.impl("slot_rowmap_ranges", &dgmc::slot_rowmap_ranges);
  m.impl("slot_rowmap_ell", &dgmc::slot_rowmap_ell);
  m.impl("slot_gather_sum", &dgmc::slot_gather_sum);
  m.impl("slot_wgrad_f32", &dgmc::slot_wgrad_f32);
  m.impl("sinkhorn_fwd", &dgmc::sinkhorn_fwd);
  m.impl("sinkhorn_bwd", &dgmc::sinkhorn_bwd);
  m.impl("sinkhorn_transport", &dgmc::sinkhorn_transport);
  m.impl("sinkhorn_transport_bwd", &dgmc::sinkhorn_transport_bwd);
}
