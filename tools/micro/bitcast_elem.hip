// Reproducer (ROCm 7.2 clang, gfx950): __builtin_bit_cast of an ext_vector_type
// element other than .x reads element 0.  Compile with --save-temps and look at
// k_elem: only one v_lshrrev/v_sub pair is emitted and the seed is splatted with
// op_sel_hi; k_whole (bit-cast of the whole vector) computes both halves.
// Found while trying a packed-f32 Jacobi phase: bit-cast the
// whole vector instead.
#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__global__ void k_elem(const f2 *in, u2 *out)
{
    const f2 x = in[threadIdx.x];
    out[threadIdx.x] = u2{__builtin_bit_cast(unsigned, x.x) >> 1, __builtin_bit_cast(unsigned, x.y) >> 1};
}

__global__ void k_whole(const f2 *in, u2 *out)
{
    out[threadIdx.x] = __builtin_bit_cast(u2, in[threadIdx.x]) >> 1u;
}
