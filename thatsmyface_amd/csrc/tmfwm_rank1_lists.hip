// The list passes (embed_kernel<b, true>: the full hybrid route over a device-side list) of the
// block sizes whose hybrid strip pass never defers (kDeferMax<b> = 0): used by the rank-1
// pre-pass's route (TMFWM_ROUTE_RANK1, tmfwm_rank1.hip) only.  Own TU: compiled in parallel.
#include "tmfwm_blocks.h"

namespace tmf {

template __global__ void embed_kernel<4, true>(EmbedArgs);
template __global__ void embed_kernel<6, true>(EmbedArgs);
template __global__ void embed_kernel<10, true>(EmbedArgs);
template __global__ void embed_kernel<12, true>(EmbedArgs);
template __global__ void embed_kernel<14, true>(EmbedArgs);
template __global__ void embed_kernel<16, true>(EmbedArgs);

}  // namespace tmf
