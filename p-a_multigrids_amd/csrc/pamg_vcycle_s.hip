// One n_split's instances of the fused V-cycle kernels (pamg_vcycle_impl.h): the Makefile builds
// this file once per n_split (-DPAMG_VC_S=1..8), so the instances compile in parallel.
#include "pamg_vcycle_impl.h"

#ifndef PAMG_VC_S
#error "build with -DPAMG_VC_S=<n_split>"
#endif
#define PAMG_VC_CAT2(a, b) a##b
#define PAMG_VC_CAT(a, b) PAMG_VC_CAT2(a, b)

namespace pamg {
hipError_t PAMG_VC_CAT(launch_vcycle_s, PAMG_VC_S)(hipStream_t s, vc::VArgs A, unsigned grid, int L, int part, int ar) {
    return launch_s<PAMG_VC_S>(s, A, grid, L, part, ar);
}
}  // namespace pamg
