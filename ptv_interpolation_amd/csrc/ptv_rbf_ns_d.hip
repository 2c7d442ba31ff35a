// ptv_rbf_ns_d.hip — k_rbf_ns instantiations for 32 row slots (ptv_rbf_ns.hpp; one
// translation unit per row-slot count so that they compile in parallel)
#include "ptv_rbf_ns.hpp"

namespace ptv {

PTV_RBF_NS_DECL(32) {
    switch (np) {
        case 1: launch_ns_t<32, 1>(ka, nvox, s, prec, pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status); break;
        case 4: launch_ns_t<32, 4>(ka, nvox, s, prec, pval, slots, ax, ay, az, qx, qy, qz, smooth, pw, mask, U, V, W, status); break;
        default: break;  // 10 monomials: NC <= 24 only (registers)
    }
}

}  // namespace ptv
