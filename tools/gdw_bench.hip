// Standalone timing of softmax_grad_dw_kernel variants (compile with -DMLAPI_GDW_EXP=<mask>, see
// the kernel source): which phase of the fused gradient costs what. B=65536, F=256, K=1000.
// Inputs are random; results are not checked (tests/test_kernels_gpu.py does that).
#ifndef MLAPI_GDW_NC
#define MLAPI_GDW_NC 1
#endif
#include "../csrc/kernels/softmax_grad_dw.hip"

#include <cstdio>
#include <vector>

using namespace mlapi;

// the harness times the fused kernel alone: the row-stats pass and the slab sums are stubbed out
namespace mlapi {
size_t softmax_rowstats_workspace(int64_t, int, int) { return 256; }
void launch_softmax_rowstats(const void*, int64_t, const void*, const float*, int64_t, int, int, int, void*, void*,
                             size_t, hipStream_t) {}
void launch_reduce_slabs_f32(const float*, int, int, float*, hipStream_t) {}
}  // namespace mlapi

int main() {
  const int64_t B = 65536;
  const int F = 256, K = 1000, ldx = F + 8;
  std::vector<uint16_t> hx((size_t)B * ldx), hw((size_t)K * F);
  uint32_t st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (uint16_t)(0x3c00 + ((st >> 16) & 0x3ff)); };
  for (auto& v : hx) v = rnd();
  for (auto& v : hw) v = rnd() ^ 0x8000 * (st & 1);
  std::vector<float> hb(K, 0.f), hrs(2 * B, 0.f);
  std::vector<int32_t> hy(B);
  for (int64_t i = 0; i < B; ++i) hy[i] = (int32_t)(i % K);
  void *dx, *dw, *db, *dy, *drs, *dws;
  const GdwLayout L = gdw_layout(B, K, F, MLAPI_GDW_NC);
  MLAPI_HIP_CHECK(hipMalloc(&dx, hx.size() * 2));
  MLAPI_HIP_CHECK(hipMalloc(&dw, hw.size() * 2));
  MLAPI_HIP_CHECK(hipMalloc(&db, K * 4));
  MLAPI_HIP_CHECK(hipMalloc(&dy, B * 4));
  MLAPI_HIP_CHECK(hipMalloc(&drs, B * 8));
  MLAPI_HIP_CHECK(hipMalloc(&dws, L.total));
  MLAPI_HIP_CHECK(hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  MLAPI_HIP_CHECK(hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  MLAPI_HIP_CHECK(hipMemcpy(db, hb.data(), K * 4, hipMemcpyHostToDevice));
  MLAPI_HIP_CHECK(hipMemcpy(dy, hy.data(), B * 4, hipMemcpyHostToDevice));
  MLAPI_HIP_CHECK(hipMemcpy(drs, hrs.data(), B * 8, hipMemcpyHostToDevice));
  GradDwArgs a{};
  a.X = (const uint16_t*)dx;
  a.ldx = ldx;
  a.W = (const uint16_t*)dw;
  a.bias = (const float*)db;
  a.y = (const int32_t*)dy;
  a.rowstat = (const float2*)drs;
  a.B = B;
  a.K = K;
  a.tiles = L.tiles;
  a.tiles_per_group = L.tiles_per_group;
  a.row_groups = L.row_groups;
  a.class_groups = L.class_groups;
  a.ldw = ldx;
  a.dw_slabs = (float*)((char*)dws + L.dw_off);
  a.stat_slabs = (float*)((char*)dws + L.stat_off);
  const dim3 grid((unsigned)(L.row_groups * L.class_groups));
  hipEvent_t e0, e1;
  MLAPI_HIP_CHECK(hipEventCreate(&e0));
  MLAPI_HIP_CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((softmax_grad_dw_kernel<8, false, MLAPI_GDW_NC>), grid, dim3(256), 0, 0, a);
  const int n = 50;
  MLAPI_HIP_CHECK(hipEventRecord(e0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL((softmax_grad_dw_kernel<8, false, MLAPI_GDW_NC>), grid, dim3(256), 0, 0, a);
  MLAPI_HIP_CHECK(hipEventRecord(e1));
  MLAPI_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  MLAPI_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  printf("nc=%d exp=%d grid=%u kernel_us=%.2f\n", MLAPI_GDW_NC, MLAPI_GDW_EXP, grid.x, ms * 1e3f / n);
  return 0;
}
