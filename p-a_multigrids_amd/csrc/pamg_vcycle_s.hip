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
    A.claim = nullptr;
    if (A.want_claim) {   // k_vc_resb's chain-placement mask: this code object's own g_chain_claim
        static unsigned *claim_ptr[64] = {};
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
            if (!claim_ptr[dev] && hipGetSymbolAddress((void **)&claim_ptr[dev], HIP_SYMBOL(g_chain_claim)) != hipSuccess)
                claim_ptr[dev] = nullptr;
            A.claim = claim_ptr[dev];
        }
    }
    return launch_s<PAMG_VC_S>(s, A, grid, L, part, ar);
}
}  // namespace pamg
