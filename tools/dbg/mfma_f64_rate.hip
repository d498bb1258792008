// Issue rate of the f64 MFMAs on gfx950: one wave per SIMD issues N MFMAs of one shape over 4
// independent accumulators; s_memtime (shader clock) around the loop gives cycles per MFMA.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_f64_rate tools/dbg/mfma_f64_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(4))) double d4_t;

template <int SHAPE>
__global__ __launch_bounds__(256) void rate_kernel(double* out, unsigned long long* cyc, int n) {
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (SHAPE == 16) {
    d4_t c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < n; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  } else {
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < n; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  }
}

int main() {
  double* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 64 * 256 * sizeof(double)) != hipSuccess || hipMalloc(&cyc, 64 * 8) != hipSuccess) return 1;
  const int n = 4096;
  for (int shape : {16, 4}) {
    for (int rep = 0; rep < 2; ++rep) {
      if (shape == 16)
        hipLaunchKernelGGL(rate_kernel<16>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      else
        hipLaunchKernelGGL(rate_kernel<4>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      unsigned long long c = 0;
      if (hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      const double per = (double)c / (4.0 * n);
      const double macs = shape == 16 ? 16 * 16 * 4 : 4 * 4 * 4 * 4;  // 4x4x4_4b: 4 blocks of 4x4x4
      std::printf("v_mfma_f64_%s: %.1f clocks per MFMA (one wave per SIMD, 4 chains) = %.1f MACs / clock\n",
                  shape == 16 ? "16x16x4" : "4x4x4_4b", per, macs / per);
    }
  }
  return 0;
}
