// Operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950, probed: A one-hot at lane p,
// B = lane + 1 -> which result lanes see which B lanes. Prints, per A lane p, the result lanes that
// came out nonzero and the B lane whose value each holds.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_f64_4x4_layout tools/dbg/mfma_f64_4x4_layout.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(double* out) {
  const int lane = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    const double a = lane == p ? 1.0 : 0.0;
    const double b = lane + 1.0;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[p * 64 + lane] = d;
  }
}

int main() {
  double* d;
  if (hipMalloc(&d, 64 * 64 * sizeof(double)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  double h[64 * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  for (int p = 0; p < 64; ++p) {
    std::printf("A lane %2d ->", p);
    for (int l = 0; l < 64; ++l)
      if (h[p * 64 + l] != 0.0) std::printf(" D%d=B%d", l, (int)h[p * 64 + l] - 1);
    std::printf("\n");
  }
  return 0;
}
