// Minimal reproducer of the round-4 "scored gather queue" fault: with ROCm 7.2
// clang, __builtin_bit_cast(float, v.y) on an ext_vector element lvalue
// compiles to element 0 (hipcc --offload-arch=gfx950 -O3 --cuda-device-only
// -S -emit-llvm: "extractelement <4 x float> %v, i64 0").  The decode kernel
// copies vector words into scalars before any bit_cast.
#include <hip/hip_runtime.h>
typedef unsigned u32x4 __attribute__((ext_vector_type(4), may_alias));
__global__ void k(const u32x4* in, float* out) {
  u32x4 v = in[threadIdx.x];
  out[threadIdx.x] = __builtin_bit_cast(float, v.y);
}
