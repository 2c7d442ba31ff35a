// ptv_knn_ka.hip — k-NN kernel instantiations for list lengths 1, 4, 8
// (split from ptv_knn.hip so that the list lengths compile in parallel)
#include "ptv_knn_impl.hpp"

namespace ptv {

#define PTV_KNN_INST(K, E)                                                                      \
    template void launch_t<K, E>(dim3, hipStream_t, const KnnKernelArgs &, const Binned &, const double *, \
                                 const double *, const double *, const double *, const double *,        \
                                 const double *, const uint8_t *, double *, double *, double *);
PTV_KNN_INST(1, false)
PTV_KNN_INST(4, false)
PTV_KNN_INST(8, false)
#undef PTV_KNN_INST

}  // namespace ptv
