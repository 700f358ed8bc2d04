// embed_kernel<8> (the benchmark's kernel, configs[1]-[3]) in a TU of its own: the
// Makefile compiles it with the max-ILP machine scheduler, which interleaves the
// independent rotation / dot-product chains of a Jacobi round (embed<8> -2 % per frame,
// measured); the other instantiations stay with the default scheduler, under which
// they keep more waves per SIMD.
#include "tmfwm_blocks.h"

namespace tmf {
template __global__ void embed_kernel<8, false>(EmbedArgs);
template __global__ void embed_kernel<8, true>(EmbedArgs);
}  // namespace tmf

#ifdef TMF_STAMPS
// phase stamps of this TU's embed_kernel<8> (its own copy of g_stamps; tools/phase_stamps.py)
extern "C" int tmfwm_debug_stamps_e8(unsigned long long *out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tmf::g_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -5;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(tmf::g_stamps), z, sizeof z) != hipSuccess) return -5;
    }
    return 0;
}
#endif
