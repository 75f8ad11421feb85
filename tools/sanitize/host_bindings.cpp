// Sanitizer build of the host runtime (csrc/runtime.cpp: tile / lane / LPT schedules,
// population sort) as its own extension module, compiled with AddressSanitizer +
// UndefinedBehaviorSanitizer by tools/sanitize/build.sh.  GPU ASan is not
// available on this pool, so the sanitizer covers the native host code.
#include <torch/extension.h>

#include <tuple>
#include <vector>

namespace mg {
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

PYBIND11_MODULE(_C_host_asan, m) {
  m.def("build_tiles", &mg::build_tiles);
  m.def("sort_by_population", &mg::sort_by_population);
  m.def("build_lanes", &mg::build_lanes, pybind11::arg("counts"), pybind11::arg("breaks"),
        pybind11::arg("window"), pybind11::arg("lmax"), pybind11::arg("order_counts") = pybind11::none());
  m.def("lpt_waves", &mg::lpt_waves);
}
