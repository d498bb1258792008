// Host-side launchers for the HIP kernels in csrc/kernels/*.hip.
// Every pointer is a device-accessible address (device memory, or host-pinned mapped memory for
// the zero-copy serving path). All launchers are asynchronous on `stream` and capture-safe
// (no allocation, no synchronization) so they can be recorded into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mlapi {

class P2PAllReduce;  // csrc/dist/p2p.h: the rank's IPC exchange for fused DP all-reduces

// Serving completion signal: instead of an event per batch (hipEventRecord + polling costs
// ~12 us launch-to-observed on MI355X, tools/launch_probe.hip), the serving kernel itself
// publishes `seq` into a host-coherent word once every block's results are out (system-scope
// release; multi-block launches elect the last block through `counter`, a device word that is
// zero between launches). The engine's completer spins on the word (~7 us). done == nullptr:
// no signal (library / test callers).
struct ServeSignal {
  uint32_t* done = nullptr;     // host-coherent, device-mapped
  uint32_t seq = 0;
  uint32_t* counter = nullptr;  // device memory, zero-initialised (multi-block kernels)
};
// Standalone signal (one wave) for kernels without a built-in one; stream order puts it after them.
void launch_serve_signal(const ServeSignal& sig, hipStream_t stream);

// ---- linear_small.hip: fused  z = x W^T + b  -> (argmax label, p_max)  for small F, K ----------
// X: [B, F] (ld = ldx elements) in dtype `dt` (F64 or F32); W: [K, F]; b: [K] (same dtype).
// out_idx: int32[B]; out_p: dtype[B]. K = rows of W (1 for binary kinds).
void launch_linear_small(int dt, const void* X, int64_t ldx, const void* W, const void* b, int64_t B, int F,
                         int K, int kind, int32_t* out_idx, void* out_p, hipStream_t stream,
                         const ServeSignal& sig = ServeSignal());

// Kernel-argument batch (linear_small.hip): a tiny serving batch travels INSIDE the kernel's
// argument block (rows + W + b), so the kernel reads nothing over the host link: the runtime
// copies the argument block into device-visible kernarg memory together with the dispatch
// packet. Only the (idx, p) results go back, written straight into host-mapped memory.
constexpr int INLINE_X_BYTES = 3072;
constexpr int INLINE_WB_BYTES = 512;
constexpr int INLINE_MAX_ROWS = 128;  // one block of <= 128 threads
struct InlineBatch {
  int32_t n, F, K, kind;
  int32_t* out_idx;
  void* out_p;
  uint32_t* done;  // ServeSignal of the batch (one block: no counter); null with `rec`
  uint32_t seq;
  // Per-row completion records (host-mapped, ServeRecord[n]); when set, each row's result AND the
  // batch's sequence number go out in ONE 16-byte store, with no fence and no done word.
  void* rec;
  // Scatter mode (combined batches of the engine's lanes): rec is a record arena and row r's record
  // goes to rec[rec_idx[r]] (each row back to its own IO thread's ring); `done` then gets the batch
  // seq from lane 0 after its record, write-through, no fence (the launcher's in-flight count only).
  int32_t rec_scatter;
  alignas(16) unsigned char wb[INLINE_WB_BYTES];  // W [K][F] then b [K] (dtype of the launch)
  alignas(16) unsigned char x[INLINE_X_BYTES];    // rows [n][F]
  alignas(16) uint32_t rec_idx[INLINE_MAX_ROWS];  // scatter mode only (only n entries are copied)
};
// One row's result as the host polls it: seq last written by the batch that produced it.
struct alignas(16) ServeRecord {
  uint32_t seq;
  int32_t idx;
  double p;
};
// Completion-record output of a serving launch: when `rec` is set, each row's (idx, p) and `seq`
// leave the kernel in one 16-byte system-scope store into rec[row] instead of out_idx / out_p.
struct RecOut {
  ServeRecord* rec = nullptr;
  uint32_t seq = 0;
};

// A queue of the caller's own that launches kernels of the serving code object by name
// (csrc/runtime/direct_dispatch.cpp: AQL packets into an HSA queue, ~0.1 us of CPU instead of
// hipLaunchKernel's ~3 us). `args`: the kernel's by-value argument block; grid in blocks.
// ordered: the kernel starts after every earlier packet of that queue has finished and its writes
// are released at kernel end (a stream's order: launches that share a workspace); unordered: it
// may overlap earlier kernels and must publish what it writes itself (write-through completion
// records). false: the kernel is not in the code object (the caller then uses hipLaunchKernel).
class KernelLauncher {
 public:
  virtual ~KernelLauncher() = default;
  virtual bool launch_kernel(const char* name, const void* args, size_t bytes, unsigned grid_x, unsigned grid_y,
                             unsigned block, bool ordered) = 0;
};
#if defined(__HIP__)  // HIP sources (both compilation passes); plain C++ includers skip it
__device__ __forceinline__ void put_record(ServeRecord* dst, uint32_t seq, int32_t idx, double p) {
  const uint64_t pb = __builtin_bit_cast(uint64_t, p);
  typedef __attribute__((ext_vector_type(4))) uint32_t rec_u32x4_t;
  const rec_u32x4_t v = {seq, (uint32_t)idx, (uint32_t)pb, (uint32_t)(pb >> 32)};
  // write-through vector store (sc0 sc1): visible to the host without a fence or a flush. The
  // s_nop: a store of more than 64 bits reads its data VGPRs after issue, so a VALU write to them
  // right behind it needs a wait state - hipcc inserts it for its own stores, never inside asm
  // (linear_wide's partials were clobbered by the next store's address computation without it)
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ void put_result(int32_t* out_idx, float* out_p, const RecOut& ro, int64_t row,
                                           int32_t idx, float p) {
  if (ro.rec != nullptr) {
    put_record(ro.rec + row, ro.seq, idx, (double)p);
  } else {
    out_idx[row] = idx;
    out_p[row] = p;
  }
}
#endif
// true if n rows of F features (and the K x F model) fit the argument block in dtype `dt`
bool linear_inline_fits(int dt, int64_t n, int F, int K);
void launch_linear_inline(int dt, const InlineBatch& a, hipStream_t stream);

// ---- gemv_binary.hip: binary LR predict, HBM-streaming GEMV + sigmoid epilogue ----------------
// X: [B, F] bf16 or f32 row-major; w: [F] same dtype; bias: scalar f32.
// out_idx: int32[B] (z > 0), out_p: f32[B] = sigmoid(|z|) (kind BINARY) or sigmoid(2|z|).
void launch_gemv_binary(int dt, const void* X, const void* w, float bias, int64_t B, int F, int kind,
                        int32_t* out_idx, float* out_p, hipStream_t stream, RecOut ro = RecOut{},
                        KernelLauncher* direct = nullptr);

// ---- gemm_softmax.hip: multiclass predict, bf16 MFMA GEMM + online softmax/argmax epilogue ----
// X: [B, F] bf16; W: [K, F] bf16; b: [K] f32. F in {32, 64, 128, 256} or a multiple of 256 (any
// width: the row-group kernel loops F in 256-feature slices). Workspace: gemm_softmax_workspace()
// (0 when the row-group kernel serves the shape).
size_t gemm_softmax_workspace(int64_t B, int K, int F);
// The automatic plan of a gemm_softmax call (host only): out = {kernel (0 16x16 tiles, 1 32x32,
// 2 row-group), 16-row tiles per wave, class splits, classes per split, row blocks}.
void gemm_softmax_plan_info(int64_t B, int K, int F, int64_t out[5]);
// Benchmark hook: force the tiles kernel's (rows-per-wave tiles, class splits) plan and the
// kernel (0 automatic, 1 tiles 16x16x32, 2 row-group, 3 tiles 32x32x16); all 0 = automatic.
void gemm_softmax_force_plan(int nt, int splits, int kernel = 0);
// Profiling hook: tiles launches write 4 s_memtime stamps per wave to this device buffer
// (tools/gemm_phase_probe.py); nullptr = off (default).
void gemm_softmax_set_stamps(void* stamps);
void launch_gemm_softmax(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                         int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes, hipStream_t stream,
                         RecOut ro = RecOut{});
// Full logits (for tests / decision_function): Z[B, K] f32.
void launch_gemm_logits(const void* X, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                        hipStream_t stream);

// Online softmax state per row for a class shard (gemm_softmax.hip MODE 4): out[B] float4 =
// {max logit, sum exp(z - max) (OvR: sum sigmoid(z)), argmax (int bits, shard-local), 0}.
// Workspace as gemm_softmax_workspace(B, K, F).
void launch_gemm_rowstate(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                          void* out_state, void* workspace, size_t ws_bytes, hipStream_t stream);

// ---- shard.hip: epilogues of sharded models ------------------------------------------------------
struct ShardOffsets {
  static constexpr int MAX = 64;
  int off[MAX];  // first class index of each shard (rank order)
};
// parts: [nparts][B] float4 row states (MODE 4), merged in shard order -> (label, p_max).
void launch_merge_rowstates(const void* parts, int nparts, int64_t B, const ShardOffsets& offs, int kind,
                            int32_t* out_idx, float* out_p, hipStream_t stream);
// Full logits Z[B, K] f32 (+ bias b[K]) -> (label, p_max) with the sklearn epilogue of `kind`.
void launch_logits_epilogue(const float* Z, const float* b, int64_t B, int K, int kind, int32_t* out_idx, float* out_p,
                            hipStream_t stream);

// ---- linear_split.hip: class-split multiclass predict for small batches (serving: B <= 32 rows)
// and for f32 models at any batch (v_mfma_f32_16x16x4_f32). X, W in dt (DT_BF16 or DT_F32), W row
// stride F (a power of two: bf16 32..512, f32 16..512), b f32 [K]. Workspace:
// linear_split_workspace(B, K) bytes, zeroed once (split-merge counters re-armed in-kernel).
// Host-merge output (serving, B <= 32): each 64-class block writes one 16-byte record per row
// {seq, argmax, m, s} (m, s: f32 bits; s = sum exp(z - m), OvR: sum sigmoid(z)) at
// rec[block * 32 + row]; the host merges the linear_split_nsplit(K) blocks in block order.
struct alignas(16) SplitRecord {
  uint32_t seq;
  int32_t bi;
  float m, s;
};
struct SplitRecOut {
  SplitRecord* rec = nullptr;
  uint32_t seq = 0;
};
bool linear_split_supported(int dt, int F);
size_t linear_split_workspace(int64_t B, int K);
// byte offset of the XCD-placement error word in the workspace (non-zero: a block of the
// XCD-local merge read a partial written on another XCD; bit x = the merging block's XCD)
size_t linear_split_xcd_err_offset();
// gemm_softmax / softmax_rowstats workspaces: byte offset of the XCD-placement error word of the
// XCD-local split merge (bit x: a merging block on XCD x read a partial written elsewhere)
size_t gemm_softmax_xcd_err_offset();
// xcd.hip: may the XCD-local split merges run on the current device? The first eager call probes
// the block -> XCD placement (1024 blocks read HW_REG_XCC_ID); inside a stream capture it answers
// the plan's default (true) without probing. xcd_placement_state: 0 not probed, 1 blocks b and b + 8k share an XCD,
// 2 off (mismatches: blocks off the plan in the probe, -1 if the probe itself failed).
bool xcd_local_allowed(hipStream_t stream);
int xcd_placement_state(int device);
int xcd_placement_mismatches(int device);
// A serving row whose XCD-local merge read a partial written on another XCD comes back with this
// label (and p = NaN) instead of a silently wrong answer; the engine fails the row and calls
// xcd_local_report_error, which switches the XCD-local protocol off for the device (the
// agent-scope protocol from the next launch on) and counts the event (xcd_local_errors).
constexpr int32_t XCD_BAD_IDX = -2;
// linear_wide: a row whose class merge waited over 1 s for a class block's state (never expected:
// the blocks of a launch are co-resident) fails with this label and p = NaN
constexpr int32_t WIDE_TIMEOUT_IDX = -3;
void xcd_local_report_error(int device);
uint64_t xcd_local_errors(int device);
// test hook: the next `launches` XCD-local launches report every merged row as misplaced
void xcd_local_inject(int launches);
void xcd_local_reset(int device);  // forget the decision: the next launch probes again
int xcd_local_take_inject();
int linear_split_nsplit(int K);
// test hook: force the XCD-local split merge on (1) / off (0), or back to MLAPI_SPLIT_XCD (-1)
void linear_split_set_xcd(int mode);
constexpr int64_t LINEAR_SPLIT_MAX_ROWS = 2048;  // rows per launch_linear_split call
// direct: launch through that queue instead of `stream` (the caller keeps every launch that shares
// the workspace on one of the two; serving completes through records, so nothing else needs the
// stream's order)
void launch_linear_split(int dt, const void* X, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K,
                         int kind, int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes,
                         hipStream_t stream, RecOut ro = RecOut(), SplitRecOut sro = SplitRecOut(),
                         KernelLauncher* direct = nullptr);

// ---- linear_wide.hip: f64-accumulating predict for wide models (linear_wide.h) ----------------
// X, W stored as f64 or f32 (dt), row stride ldx >= plan.ldx with the columns F..ldx zero in both;
// b: f64 [K]. Every kind (binary kinds: K = 1). Accumulation in f64 on the matrix cores
// (v_mfma_f64_16x16x4_f64), so f32 storage loses nothing beyond the f32 rounding of its inputs.
// Grid: plan.ncb 16-class blocks x plan.nfs feature splits x ceil(B / 32) row groups.
struct WidePlan {
  int ncb = 0;     // 16-class blocks
  int nfs = 0;     // feature splits over blocks (their partial logits summed by the last arriver)
  int ldx = 0;     // padded row width the kernel reads (multiple of the split unit)
  int fsteps = 0;  // steps per wave per split
};
WidePlan linear_wide_plan(int dt, int F, int K);
// measurement hook: later launches stop early (1: after the MFMA loop, 2: before the class merge)
void linear_wide_set_probe(int probe);
// measurement: per-block wall-clock timeline of the wide kernel (8 x u64 per block, device memory;
// nullptr = off)
void linear_wide_set_trace(void* trace);
// workspace (zeroed once; tickets are re-armed in-kernel) for up to B rows
size_t linear_wide_workspace(int64_t B, int dt, int F, int K);
// Host class merge (serving, multiclass, B <= 32): block cb writes for row r two 16-byte units at
// rec[(cb * 32 + r) * 2 + {0, 1}] = {seq, argmax, m (f64)}, {seq, 0, s (f64)} and the host merges
// the plan.ncb blocks in block order (split_merge.h, merge_wide_records).
struct alignas(16) WideRecord {
  uint32_t seq;
  int32_t v;  // argmax (unit 0), 0 (unit 1)
  double x;   // m (unit 0), s (unit 1)
};
struct WideRecOut {
  WideRecord* rec = nullptr;
  uint32_t seq = 0;
};
// ws_private: no other launch in flight uses this workspace (the engine gives every batch slot its
// own), so a direct-dispatched launch may overlap the ones before it (unordered packet).
void launch_linear_wide(int dt, const void* X, int64_t ldx, const void* W, const double* b, int64_t B, int F, int K,
                        int kind, int32_t* out_idx, double* out_p, void* workspace, size_t ws_bytes, hipStream_t stream,
                        RecOut ro = RecOut(), WideRecOut hro = WideRecOut(), KernelLauncher* direct = nullptr,
                        bool ws_private = false);

// Multiclass training row stats (gemm_softmax.hip MODE 2), X_aug = [X | 0.. | 1 | 0 x 7] bf16
// read through its row stride ldx (the first F columns); W: [K, F] bf16; b: [K] f32.
// MODE 2 alone: rowstat_out[B] = {logsumexp (OvR: max + log sum sigmoid), argmax bits} per row.
size_t softmax_rowstats_workspace(int64_t B, int K, int F);
void launch_softmax_rowstats(const void* X_aug, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K,
                             int kind, void* rowstat_out, void* workspace, size_t ws_bytes, hipStream_t stream);
// Fused gradient (softmax_grad_dw.hip): row stats, then G and dW_aug = G^T X_aug in one MFMA kernel
// (G never touches HBM), then the deterministic slab reductions. dW_out: [K, F + 8] f32 (column F
// = intercept gradient, F+1.. = 0); stats_out = [loss_sum, n_correct]. F in {128, 256, 512}
// (narrower models are zero-padded by the caller), ldx = F + 8. Workspace:
// softmax_grad_dw_workspace(B, K, F) bytes, zeroed once.
bool softmax_grad_dw_supported(int F);
void softmax_grad_dw_force_plan(int row_groups, int nc);  // benchmark hook (0 = automatic)
size_t softmax_grad_dw_workspace(int64_t B, int K, int F);
// Optional SGD update fused into the final slab sum (one replica: no all-reduce between them):
// params [K, cols] -= lr * (dW / N + l2 * params[:, :pen_cols]) with momentum, refreshing the bf16 /
// f32 shadow copies the forward reads - sgd_update_2d's arithmetic, one launch fewer.
struct Sgd2D {
  float* params = nullptr;
  float* mom = nullptr;
  uint16_t* shadow_w = nullptr;
  float* shadow_b = nullptr;
  int cols = 0, pen_cols = 0;
  float lr = 0.f, inv_n = 0.f, l2 = 0.f, momentum = 0.f;
};
// With `dp`, the final slab sum also performs the DP all-reduce in-kernel (p2p_device.h) before the
// fused update: 3 launches per multiclass step at any world size.
void launch_softmax_grad_dw(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y,
                            int64_t B, int F, int K, int kind, float* dW_out, float* stats_out, void* workspace,
                            size_t ws_bytes, hipStream_t stream, const Sgd2D* update = nullptr,
                            P2PAllReduce* dp = nullptr, int dp_timeout_ms = 0);

// The deterministic final sum of [nslabs][K][F_aug] dW slabs + [nstat][2] stat slabs, with the
// optional fused SGD update and in-kernel DP exchange (softmax_grad_dw.hip's last launch).
void launch_gdw_reduce(const float* slabs, int nslabs, int K, int F_aug, float* dW_out, const float* stat_slabs,
                       int nstat, float* stats_out, const Sgd2D* update, P2PAllReduce* dp, int dp_timeout_ms,
                       hipStream_t stream);
// Full logits Z [B, K] f32 of X [B, F] (row stride ldx) through the row-group kernel.
// Row stats + training G in one launch (row-group kernel MODE 5): G = softmax(z) - onehot(y) (OvR:
// sigmoid(z) - onehot) as bf16 [B][Kp] (zero columns K..Kp-1) and per-block {loss, correct} in
// stat_slabs[softmax_rows_g_blocks(B)][2]. F: a multiple of 256 (or a power of two <= 256). Zs
// (optional, [B][Kp] f32): the first pass stores its logits there and the second reads them back
// instead of recomputing them; null recomputes.
int softmax_rows_g_blocks(int64_t B, int F, int K);
// true: launch_softmax_rows_g keeps the logits in registers (softmax_rows_g2_kernel) and never
// touches Zs, so callers need no [B][Kp] f32 buffer for it
bool softmax_rows_g_keeps_logits(int64_t B, int F, int K, int Kp);
// measurement / tests: -1 = MLAPI_ROWS_G2 (default on), 0 = the XLDS kernel + logits buffer, 1 = on
void gemm_softmax_set_rows_g2(int on);
// bytes of the fragment-ordered W copy the register-resident G kernel reads (0: it does not apply);
// pass such a buffer (16-byte aligned) as w_packed, or null for the row-major reads
size_t softmax_rows_g_wpack_bytes(int64_t B, int F, int K, int Kp);
// measurement / tests: -1 = MLAPI_G2_PACKED (default on), 0 = row-major W reads, 1 = packed
void gemm_softmax_set_w_packed(int on);
void launch_softmax_rows_g(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y, int64_t B,
                           int F, int K, int kind, uint16_t* G, int Kp, float* stat_slabs, float* Zs,
                           void* w_packed, hipStream_t stream);
void launch_gemm_logits_ld(const void* X, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                           hipStream_t stream);
// Multiclass training gradient for wide models (softmax_grad_wide.hip): F a multiple of 256 above
// 512 (X_aug row stride F + 8). Row stats and logits by the row-group kernel, G = P - Y (bf16) with
// the loss / correct stats, dW slabs = G^T X_aug by an MFMA kernel (LDS tiles read through
// ds_read_b64_tr_b16), then launch_gdw_reduce. Workspace: softmax_grad_wide_workspace bytes.
bool softmax_grad_wide_supported(int F);
void softmax_grad_wide_set_zbuf(int mode);  // measurement / test hook: -1 env default, 0 recompute, 1 keep logits
size_t softmax_grad_wide_workspace(int64_t B, int K, int F);
void launch_softmax_grad_wide(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y,
                              int64_t B, int F, int K, int kind, float* dW_out, float* stats_out, void* workspace,
                              size_t ws_bytes, hipStream_t stream, const Sgd2D* update = nullptr,
                              P2PAllReduce* dp = nullptr, int dp_timeout_ms = 0);

// ---- train kernels (train.hip) -----------------------------------------------------------------
// Binary logistic regression, one pass over X: accumulates grad (F w-entries, 1 bias) and stats
// [loss_sum, n_correct] into per-block slabs, then reduce_slabs() folds them into out[F + 3]:
// out = [gW(F) | gb | loss_sum | n_correct]  (sums over the batch, not means).
size_t train_binary_workspace(int64_t B, int F);
void train_binary_set_max_blocks(int n);  // benchmark hook: grid cap of the gradient kernel (0 = default)
void launch_train_binary_grad(int dt, const void* X, const float* y, const float* w, float bias_unused,
                              const float* bptr, int64_t B, int F, float* out, void* workspace, size_t ws_bytes,
                              hipStream_t stream);
// Fused step: gradient (as above, into grad_out) + deterministic reduce + SGD update of params =
// [w (F) | b] in place: 2 launches. With `dp` (the rank's P2P exchange, csrc/dist/p2p.h) the
// data-parallel all-reduce runs inside the reduce launch (p2p_device.h): still 2 launches per step
// at any world size, and world = 1 runs the same kernels. inv_n = 1 / global batch.
void launch_train_binary_step(int dt, const void* X, const float* y, float* params, float* mom, int64_t B, int F,
                              float* grad_out, void* workspace, size_t ws_bytes, float lr, float inv_n, float l2,
                              float momentum, hipStream_t stream, P2PAllReduce* dp = nullptr, int dp_timeout_ms = 0);
// Small multiclass / binary (F*K <= 1024): fp64 or fp32, exact loss+grad of sklearn's objective
// terms. out = [gW (K*F, row-major) | gb (K) | loss_sum | n_correct].
size_t train_small_workspace(int64_t B, int F, int K);
void launch_train_small_grad(int dt, const void* X, const int32_t* y, const void* W, const void* b, int64_t B,
                             int F, int K, int kind, void* out, void* workspace, size_t ws_bytes,
                             hipStream_t stream);
// SGD (+momentum) update: p -= lr * (g * inv_n + l2 * p) for the first n_penalized entries,
// p -= lr * g * inv_n for the rest (intercepts are not penalized, like sklearn).
void launch_sgd_update(float* params, const float* grad, float* momentum_buf, int64_t n, int64_t n_penalized,
                       float lr, float inv_n, float l2, float momentum, hipStream_t stream);

// Deterministic column sums of [nslabs][width] f32 partial slabs -> out[width].
void launch_reduce_slabs_f32(const float* slabs, int nslabs, int width, float* out, hipStream_t stream);
// SGD step on a row-major [rows, cols] f32 matrix W_aug = [W | b | pad] whose first pen_cols
// columns are L2-penalized (the intercept column is not); optionally refreshes in the same pass the
// copies the next forward reads: shadow_w = bf16 W [rows, pen_cols], shadow_b = f32 column pen_cols.
void launch_sgd_update_2d(float* params, const float* grad, float* momentum_buf, int64_t rows, int cols,
                          int pen_cols, float lr, float inv_n, float l2, float momentum, uint16_t* shadow_w,
                          float* shadow_b, hipStream_t stream);

// ---- pack.hip ----------------------------------------------------------------------------------
void launch_cast(int src_dt, const void* src, int dst_dt, void* dst, int64_t n, hipStream_t stream);

}  // namespace mlapi
