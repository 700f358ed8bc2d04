// embed_kernel<8> (the benchmark's kernel, configs[1]-[3]) in a TU of its own: the
// Makefile compiles it with the max-ILP machine scheduler, which interleaves the
// independent rotation / dot-product chains of a Jacobi round (embed<8> -2 % per frame,
// measured); the other instantiations stay with the default scheduler, under which
// they keep more waves per SIMD.
#include "tmfwm_blocks.h"

namespace tmf {
template __global__ void embed_kernel<8>(EmbedArgs);
}  // namespace tmf
