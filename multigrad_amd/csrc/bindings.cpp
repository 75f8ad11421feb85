// Python bindings for the multigrad_amd native extension (_C).
#include <torch/extension.h>

#include <tuple>
#include <string>
#include <vector>

namespace mg {
// smf.hip
int smf_padded_bins(int64_t nb);
int64_t smf_fwd_max_blocks(int64_t nb, bool log_sigma, bool has_pop, bool rel_tail);
void smf_forward(torch::Tensor x, c10::optional<torch::Tensor> pop, torch::Tensor theta,
                 std::vector<double> edges, std::vector<double> scale, bool log_sigma,
                 int64_t begin, int64_t end, torch::Tensor slab, int64_t nblocks, bool rel_tail,
                 std::string exchange);
void smf_slab_reduce(torch::Tensor slab, int64_t nrows, std::vector<double> edges,
                     std::vector<double> scale, torch::Tensor out);
void smf_edge_weights(torch::Tensor g, std::vector<double> edges, std::vector<double> scale,
                      torch::Tensor h);
void smf_logmse(torch::Tensor S, torch::Tensor target, double eps, std::vector<double> edges,
                std::vector<double> scale, torch::Tensor loss, torch::Tensor g_out,
                torch::Tensor h);
void smf_vjp(torch::Tensor x, c10::optional<torch::Tensor> pop, torch::Tensor theta,
             torch::Tensor tiles, int64_t tile_begin, int64_t tile_end, torch::Tensor h,
             std::vector<double> edges, std::vector<double> scale, bool log_sigma,
             torch::Tensor grad, torch::Tensor partials, torch::Tensor giant,
             std::string exchange);
int64_t smf_fwd_lanes_max_blocks(int64_t nb, bool log_sigma, bool rel_tail, bool resid);
void smf_lanes_pack(torch::Tensor xs, torch::Tensor slot_src, torch::Tensor slot_len,
                    torch::Tensor group_base, torch::Tensor group_len, torch::Tensor xi);
int64_t smf_forward_lanes(torch::Tensor xi, torch::Tensor slot_pop, torch::Tensor group_base,
                       torch::Tensor group_len, torch::Tensor fwd_order, torch::Tensor theta,
                       std::vector<double> edges,
                       std::vector<double> scale, bool log_sigma, int64_t g0, int64_t g1,
                       torch::Tensor slab, int64_t nblocks, bool rel_tail,
                       c10::optional<torch::Tensor> resid,
                       c10::optional<torch::Tensor> wave_order,
                       c10::optional<torch::Tensor> wave_start,
                       c10::optional<torch::Tensor> queues,
                       c10::optional<std::vector<torch::Tensor>> update,
                       std::vector<double> update_scalars,
                       std::vector<torch::Tensor> epi_tensors, std::vector<double> epi_scalars,
                       std::vector<int64_t> epi_peers, bool per_edge);
void smf_vjp_lanes(torch::Tensor slot_pop, torch::Tensor slot_part, torch::Tensor theta,
                   torch::Tensor h, torch::Tensor resid, int64_t s0, int64_t s1,
                   std::vector<double> scale, bool log_sigma, torch::Tensor grad,
                   torch::Tensor partials, torch::Tensor giant);
void smf_vjp_adam_lanes(torch::Tensor slot_pop, torch::Tensor slot_part, torch::Tensor theta,
                        torch::Tensor h, torch::Tensor resid, int64_t s0, int64_t s1,
                        std::vector<double> scale, bool log_sigma, torch::Tensor m,
                        torch::Tensor v, int64_t unit_offset, torch::Tensor step,
                        int64_t host_step, double lr, double b1, double b2, double eps,
                        c10::optional<torch::Tensor> traj, int64_t traj_stride);
torch::Tensor smf_fwd_trace();
void smf_vjp_lanes_rc(torch::Tensor xi, torch::Tensor slot_idx, torch::Tensor slot_part,
                      torch::Tensor group_base, torch::Tensor group_len, torch::Tensor theta,
                      torch::Tensor h, std::vector<double> edges, std::vector<double> scale,
                      bool log_sigma, int64_t g0, int64_t g1, torch::Tensor grad,
                      torch::Tensor partials, torch::Tensor giant);
void smf_epilogue(torch::Tensor slab, int64_t nrows, std::vector<double> edges,
                  std::vector<double> scale, torch::Tensor target, double eps, torch::Tensor S,
                  torch::Tensor loss, torch::Tensor h, std::vector<int64_t> peers, int64_t rank,
                  c10::optional<torch::Tensor> seq, c10::optional<torch::Tensor> err,
                  double timeout_s, c10::optional<torch::Tensor> advance);
int64_t smf2_max_bins();
int64_t smf2_fwd_max_blocks(int64_t nb, bool log_sigma);
void smf2_forward(torch::Tensor x, torch::Tensor theta, std::vector<double> edges,
                  std::vector<double> scale, bool log_sigma, torch::Tensor slab, int64_t nblocks);
void smf2_step(torch::Tensor slab, int64_t nrows, std::vector<double> edges, std::vector<double> scale,
               bool log_sigma, std::vector<torch::Tensor> state, std::vector<double> scalars,
               std::vector<int64_t> peers, int64_t rank, c10::optional<torch::Tensor> seq,
               c10::optional<torch::Tensor> err, int64_t mode);
void smf2_loop(torch::Tensor x, std::vector<double> edges, std::vector<double> scale, bool log_sigma,
               std::vector<torch::Tensor> state, std::vector<double> scalars,
               std::vector<int64_t> peers, int64_t rank, c10::optional<torch::Tensor> seq,
               c10::optional<torch::Tensor> err, int64_t steps);
// xgmi.hip
int64_t xgmi_alloc(int64_t bytes);
torch::Tensor xgmi_tensor(int64_t ptr, int64_t numel);
void xgmi_twoshot(std::vector<int64_t> gbufs, std::vector<int64_t> tbufs, std::vector<int64_t> flags,
                  int64_t rank, int64_t lo, int64_t n, int64_t total, int64_t mode,
                  c10::optional<torch::Tensor> u, c10::optional<torch::Tensor> m,
                  c10::optional<torch::Tensor> v, c10::optional<torch::Tensor> blo,
                  c10::optional<torch::Tensor> bhi, c10::optional<torch::Tensor> kind,
                  c10::optional<torch::Tensor> traj, torch::Tensor step, torch::Tensor seq,
                  torch::Tensor err, std::vector<double> scalars);
pybind11::bytes xgmi_twoshot_pack(std::vector<int64_t> gbufs, std::vector<int64_t> tbufs,
                                  std::vector<int64_t> flags, int64_t rank, int64_t lo, int64_t n,
                                  int64_t total, int64_t mode, c10::optional<torch::Tensor> u,
                                  c10::optional<torch::Tensor> m, c10::optional<torch::Tensor> v,
                                  c10::optional<torch::Tensor> blo, c10::optional<torch::Tensor> bhi,
                                  c10::optional<torch::Tensor> kind, c10::optional<torch::Tensor> traj,
                                  torch::Tensor step, torch::Tensor seq, torch::Tensor err,
                                  std::vector<double> scalars);
void xgmi_twoshot_launch_packed(std::string packed);
int64_t xgmi_twoshot_flag_bytes();
pybind11::bytes xgmi_handle(int64_t base);
int64_t xgmi_open(pybind11::bytes handle);
void xgmi_close(int64_t ptr);
void xgmi_zero(int64_t base, int64_t bytes);
void xgmi_free(int64_t ptr);
void xgmi_allreduce(torch::Tensor x, std::vector<int64_t> peers, int64_t rank, torch::Tensor seq,
                    torch::Tensor err, double timeout_s);
void xgmi_allreduce_wide(torch::Tensor x, int64_t nsum, int64_t nmax, std::vector<int64_t> peers,
                         int64_t rank, torch::Tensor seq, torch::Tensor err, double timeout_s);
int64_t xgmi_wide_region_bytes();
std::string device_pci_bus_id();
void xgmi_a2a_pull(std::vector<int64_t> src_ptrs, std::vector<int64_t> counts,
                   std::vector<int64_t> dst_offs, torch::Tensor out);
// adam.hip
void fused_adam(torch::Tensor u, torch::Tensor m, torch::Tensor v, torch::Tensor g,
                c10::optional<torch::Tensor> p, c10::optional<torch::Tensor> lo,
                c10::optional<torch::Tensor> hi, c10::optional<torch::Tensor> kind,
                torch::Tensor step, double lr, double b1, double b2, double eps, bool legacy,
                c10::optional<torch::Tensor> traj, int64_t traj_stride, int64_t host_step);
// lbfgs.hip
void multi_dot(torch::Tensor A, int64_t nrows, std::vector<torch::Tensor> B, int64_t n,
               torch::Tensor out, torch::Tensor workspace);
int64_t multi_dot_workspace(int64_t nrows, int64_t n);
void lincomb(torch::Tensor H, int64_t nrows, torch::Tensor coef, double alpha,
             c10::optional<torch::Tensor> x, int64_t n, torch::Tensor y);
// runtime.cpp
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, int64_t>
build_tiles(torch::Tensor counts, std::vector<int64_t> breaks, int64_t tile_halos,
            int64_t tile_pops);
std::tuple<torch::Tensor, torch::Tensor> sort_by_population(torch::Tensor pop, int64_t npop);
std::vector<torch::Tensor> build_lanes(torch::Tensor counts, std::vector<int64_t> breaks,
                                       int64_t window, int64_t lmax,
                                       c10::optional<torch::Tensor> order_counts);
std::vector<torch::Tensor> lpt_waves(torch::Tensor group_len, torch::Tensor fwd_order,
                                     int64_t g0, int64_t g1, int64_t nwaves, double overhead);
}  // namespace mg

#ifndef MG_BUILD_HASH
#define MG_BUILD_HASH "unknown"
#endif
#ifndef MG_BUILD_ARCH
#define MG_BUILD_ARCH "unknown"
#endif

PYBIND11_MODULE(_C, m) {
  m.doc() = "multigrad_amd native extension (gfx950 HIP kernels + host runtime)";
  m.def("build_info", []() {
    pybind11::dict d;
    d["source_hash"] = MG_BUILD_HASH;
    d["offload_arch"] = MG_BUILD_ARCH;
    d["compiled"] = __DATE__ " " __TIME__;
    return d;
  });
  m.def("smf_padded_bins", &mg::smf_padded_bins);
  m.def("smf_forward", &mg::smf_forward, pybind11::arg("x"), pybind11::arg("pop"),
        pybind11::arg("theta"), pybind11::arg("edges"), pybind11::arg("scale"),
        pybind11::arg("log_sigma"), pybind11::arg("begin"), pybind11::arg("end"),
        pybind11::arg("slab"), pybind11::arg("nblocks"), pybind11::arg("rel_tail"),
        pybind11::arg("exchange") = std::string());
  m.def("smf_fwd_max_blocks", &mg::smf_fwd_max_blocks);
  m.def("smf_slab_reduce", &mg::smf_slab_reduce);
  m.def("smf_edge_weights", &mg::smf_edge_weights);
  m.def("smf_logmse", &mg::smf_logmse);
  m.def("smf_vjp", &mg::smf_vjp, pybind11::arg("x"), pybind11::arg("pop"), pybind11::arg("theta"),
        pybind11::arg("tiles"), pybind11::arg("tile_begin"), pybind11::arg("tile_end"),
        pybind11::arg("h"), pybind11::arg("edges"), pybind11::arg("scale"),
        pybind11::arg("log_sigma"), pybind11::arg("grad"), pybind11::arg("partials"),
        pybind11::arg("giant"), pybind11::arg("exchange") = std::string());
  m.def("smf_fwd_lanes_max_blocks", &mg::smf_fwd_lanes_max_blocks);
  m.def("smf_lanes_pack", &mg::smf_lanes_pack);
  m.def("smf_forward_lanes", &mg::smf_forward_lanes, pybind11::arg("xi"), pybind11::arg("slot_pop"),
        pybind11::arg("group_base"), pybind11::arg("group_len"), pybind11::arg("fwd_order"),
        pybind11::arg("theta"), pybind11::arg("edges"), pybind11::arg("scale"),
        pybind11::arg("log_sigma"), pybind11::arg("g0"), pybind11::arg("g1"), pybind11::arg("slab"),
        pybind11::arg("nblocks"), pybind11::arg("rel_tail"), pybind11::arg("resid") = pybind11::none(),
        pybind11::arg("wave_order") = pybind11::none(), pybind11::arg("wave_start") = pybind11::none(),
        pybind11::arg("queues") = pybind11::none(), pybind11::arg("update") = pybind11::none(),
        pybind11::arg("update_scalars") = std::vector<double>(),
        pybind11::arg("epi_tensors") = std::vector<torch::Tensor>(),
        pybind11::arg("epi_scalars") = std::vector<double>(),
        pybind11::arg("epi_peers") = std::vector<int64_t>(), pybind11::arg("per_edge") = false);
  m.def("lpt_waves", &mg::lpt_waves);
  m.def("smf_vjp_lanes", &mg::smf_vjp_lanes);
  m.def("smf_vjp_adam_lanes", &mg::smf_vjp_adam_lanes);
  m.def("smf_fwd_trace", &mg::smf_fwd_trace);
  m.def("smf_vjp_lanes_rc", &mg::smf_vjp_lanes_rc);
  m.def("smf_epilogue", &mg::smf_epilogue, pybind11::arg("slab"), pybind11::arg("nrows"),
        pybind11::arg("edges"), pybind11::arg("scale"), pybind11::arg("target"), pybind11::arg("eps"),
        pybind11::arg("S"), pybind11::arg("loss"), pybind11::arg("h"), pybind11::arg("peers"),
        pybind11::arg("rank"), pybind11::arg("seq"), pybind11::arg("err"), pybind11::arg("timeout_s"),
        pybind11::arg("advance") = pybind11::none());
  m.def("smf2_max_bins", &mg::smf2_max_bins);
  m.def("smf2_fwd_max_blocks", &mg::smf2_fwd_max_blocks);
  m.def("smf2_forward", &mg::smf2_forward);
  m.def("smf2_step", &mg::smf2_step);
  m.def("smf2_loop", &mg::smf2_loop);
  m.def("xgmi_alloc", &mg::xgmi_alloc, pybind11::arg("bytes") = 0);
  m.def("xgmi_tensor", &mg::xgmi_tensor);
  m.def("xgmi_twoshot", &mg::xgmi_twoshot);
  m.def("xgmi_twoshot_pack", &mg::xgmi_twoshot_pack);
  m.def("xgmi_twoshot_launch_packed", &mg::xgmi_twoshot_launch_packed);
  m.def("xgmi_twoshot_flag_bytes", &mg::xgmi_twoshot_flag_bytes);
  m.def("xgmi_handle", &mg::xgmi_handle);
  m.def("xgmi_open", &mg::xgmi_open);
  m.def("xgmi_close", &mg::xgmi_close);
  m.def("xgmi_zero", &mg::xgmi_zero, pybind11::arg("base"), pybind11::arg("bytes") = 0);
  m.def("xgmi_free", &mg::xgmi_free);
  m.def("xgmi_allreduce", &mg::xgmi_allreduce);
  m.def("xgmi_allreduce_wide", &mg::xgmi_allreduce_wide);
  m.def("xgmi_wide_region_bytes", &mg::xgmi_wide_region_bytes);
  m.def("device_pci_bus_id", &mg::device_pci_bus_id);
  m.def("xgmi_a2a_pull", &mg::xgmi_a2a_pull);
  m.def("fused_adam", &mg::fused_adam, pybind11::arg("u"), pybind11::arg("m"), pybind11::arg("v"),
        pybind11::arg("g"), pybind11::arg("p"), pybind11::arg("lo"), pybind11::arg("hi"),
        pybind11::arg("kind"), pybind11::arg("step"), pybind11::arg("lr"), pybind11::arg("b1"),
        pybind11::arg("b2"), pybind11::arg("eps"), pybind11::arg("legacy"), pybind11::arg("traj"),
        pybind11::arg("traj_stride"), pybind11::arg("host_step") = -1);
  m.def("multi_dot", &mg::multi_dot);
  m.def("multi_dot_workspace", &mg::multi_dot_workspace);
  m.def("lincomb", &mg::lincomb);
  m.def("build_tiles", &mg::build_tiles);
  m.def("sort_by_population", &mg::sort_by_population);
  m.def("build_lanes", &mg::build_lanes, pybind11::arg("counts"), pybind11::arg("breaks"),
        pybind11::arg("window"), pybind11::arg("lmax"), pybind11::arg("order_counts") = pybind11::none());
}
