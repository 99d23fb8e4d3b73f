// Host-side launch API of the tensorframes_amd HIP kernel library (gfx950 / CDNA4).
//
// These functions are torch-free: raw device pointers + hipStream_t. Each one
// checks the shapes it is handed against what its grid assumes before it
// launches (a bad launch can fault the whole node).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

#include "../common.h"

namespace tfa {
namespace k {

constexpr int kMaxRank = 8;

void check_launch(const char* what);

// ------------------------------------------------------------ elementwise
enum class BinOp : int {
  ADD, SUB, MUL, DIV, FLOORDIV, FLOORMOD, TRUNCMOD, MAX, MIN, POW, SQDIFF,
  EQ, NE, LT, LE, GT, GE, LAND, LOR, ATAN2, DIVNONAN,
};
enum class UnOp : int {
  NEG, ABS, SQUARE, SQRT, RSQRT, EXP, LOG, LOG1P, EXPM1, RECIP, RELU, RELU6, ELU, SELU,
  SIGMOID, TANH, SOFTPLUS, SOFTSIGN, FLOOR, CEIL, ROUND, SIGN, SIN, COS, TAN, NOT, IDENTITY,
  ERF, ISNAN, ISINF, ISFINITE,
};

// Broadcast descriptor: output dims and per-operand element strides (0 on broadcast dims).
struct Bcast {
  int rank = 0;
  int64_t dims[kMaxRank];
  int64_t sa[kMaxRank];
  int64_t sb[kMaxRank];
  int64_t sc[kMaxRank];  // third operand (Select)
};

// out = op(a, b). mode: 0 same-shape contiguous, 1 b scalar, 2 a scalar,
// 3 row-broadcast (b is [inner], a is [n/inner, inner]), 4 general broadcast.
void binary(BinOp op, DType dt, const void* a, const void* b, void* out, int64_t n, int mode,
            int64_t inner, const Bcast* bc, hipStream_t s);
// out_dtype is BOOL for comparisons/logical ops.
void unary(UnOp op, DType dt, const void* x, void* y, int64_t n, hipStream_t s);
void cast(DType from, DType to, const void* x, void* y, int64_t n, hipStream_t s);
void select(DType dt, const void* cond, const void* a, const void* b, void* out, int64_t n,
            const Bcast& bc, hipStream_t s);
void fill(DType dt, void* out, int64_t n, double value, hipStream_t s);
void range(DType dt, void* out, int64_t n, double start, double delta, hipStream_t s);


// ------------------------------------------------------------ reductions
enum class RedOp : int { SUM, PROD, MIN, MAX, MEAN, ALL, ANY };
// x viewed as [outer, r, inner] -> y [outer, inner]. workspace: see reduce_workspace_bytes.
size_t reduce_workspace_bytes(DType dt, int64_t outer, int64_t r, int64_t inner);
void reduce(RedOp op, DType dt, const void* x, void* y, int64_t outer, int64_t r, int64_t inner,
            void* workspace, hipStream_t s);
// arg-reduce over r of [outer, r, inner]; out int32 or int64
void argreduce(bool is_min, DType dt, DType out_dt, const void* x, void* y, int64_t outer,
               int64_t r, int64_t inner, hipStream_t s);
// softmax / log-softmax over the last dim of [rows, cols]
void softmax(DType dt, bool log, const void* x, void* y, int64_t rows, int64_t cols, hipStream_t s);
// top-k along the last dim of [rows, cols]: values (dt) + indices (int32), sorted descending
void topk(DType dt, const void* x, void* vals, int32_t* idx, int64_t rows, int64_t cols, int k,
          hipStream_t s);
// segmented reductions: rows of x [n, inner] with segment ids (sorted or not) into [nseg, inner]
// ---- one-shot all-reduce over IPC-mapped peer buffers (oneshot.hip)
constexpr int kOneShotMaxRanks = 8;
constexpr size_t kOneShotSlotBytes = 64 << 10;                     // largest payload
constexpr size_t kOneShotFlagOffset = 2 * kOneShotSlotBytes;       // 2 slots x 8 ranks u32
constexpr size_t kOneShotErrOffset = kOneShotFlagOffset + 2 * 8 * 4;  // timeout word
constexpr size_t kOneShotBufBytes = kOneShotErrOffset + 256;
struct OneShotPeers {
  void* buf[kOneShotMaxRanks];  // every rank's buffer, mapped into this process ([rank] = own)
};
// timeout_us bounds every flag wait (a missing peer sets the error word)
void oneshot_all_reduce(RedOp op, DType dt, const void* in, void* out, int64_t n, int rank, int world,
                        const OneShotPeers& p, uint32_t epoch, uint64_t timeout_us, hipStream_t s);
// fault injection: one wave that spins for `us` microseconds (at most 60 s) on
// the device's realtime counter, then exits; work queued behind it on `s`
// waits (a stalled peer / slow rank, for the collective timeout tests)
void device_stall(uint64_t us, hipStream_t s);

size_t unsorted_segment_workspace_bytes(RedOp op, DType dt, int64_t n, int64_t inner, int64_t nseg);
void unsorted_segment_reduce(RedOp op, DType dt, DType idt, const void* x, const void* ids,
                             void* y, int64_t n, int64_t inner, int64_t nseg, void* workspace,
                             hipStream_t s);
// segmented reduce with CSR offsets over contiguous rows (deterministic)
void segment_reduce_csr(RedOp op, DType dt, const void* x, const int64_t* offsets, void* y,
                        int64_t nseg, int64_t inner, hipStream_t s);

// ------------------------------------------------------------ groupBy (groupby.hip)
// keys [n] -> ids [n] (group of each row, groups in ascending key order) and
// uniq (first nseg entries: the distinct keys, ascending); returns nseg
// (synchronises the stream once to read it).
size_t factorize_workspace_bytes(DType dt, int64_t n);
int64_t factorize(DType dt, const void* keys, int64_t n, int64_t* ids, void* uniq, void* workspace,
                  size_t workspace_size, hipStream_t s);
// per-row 64-bit key hash (accumulate: combine with the hash already in h)
void key_hash(DType dt, const void* keys, int64_t n, uint64_t* h, bool accumulate, hipStream_t s);
void hash_mod(const uint64_t* h, int64_t n, int64_t world, int64_t* dest, hipStream_t s);
// string keys as W big-endian words (sign-flipped) + length, column-major [W+1][n]
void string_words(const int64_t* offs, const uint8_t* data, int64_t n, int W, int64_t* out, hipStream_t s);
// bounded-width string keys: [2][n] int64 = (sign-flipped big-endian word 0,
// tag = length for keys <= 8 bytes, else 9 + 62-bit hash); string_verify sets
// flag[0] when a row's bytes differ from its group representative's
void string_key_hash(const int64_t* offs, const uint8_t* data, int64_t n, int64_t* out, hipStream_t s);
void string_verify(const int64_t* offs, const uint8_t* data, const int64_t* ids, const int64_t* rep, int64_t n,
                   int* flag, hipStream_t s);
uint64_t string_key_hash_host(const uint8_t* p, int64_t len);  // the same hash on the host
// rows idx of a string column: lens[g] = length of row idx[g]; gather_bytes
// copies them to out at new_offs (the exclusive scan of lens)
void string_lens(const int64_t* offs, const int64_t* idx, int64_t n, int64_t* lens, hipStream_t s);
void gather_bytes(const uint8_t* data, const int64_t* offs, const int64_t* idx, const int64_t* new_offs, int64_t n,
                  uint8_t* out, hipStream_t s);
// ids [n] in [0, nseg) -> rows ordered by segment (stable) perm [n] and CSR
// offsets [nseg + 1]; out-of-range ids are dropped
size_t segment_csr_workspace_bytes(int64_t n, int64_t nseg);
void segment_csr(DType idt, const void* ids, int64_t n, int64_t nseg, int64_t* perm, int64_t* offsets,
                 void* workspace, size_t workspace_size, hipStream_t s);
// segment g = rows perm[offsets[g] .. offsets[g+1]) of x [*, inner] -> y [nseg, inner] (deterministic)
void segment_reduce_perm(RedOp op, DType dt, const void* x, const int64_t* perm, const int64_t* offsets, void* y,
                         int64_t nseg, int64_t inner, hipStream_t s);
// rep[g] = some row of group g (ids in [0, nseg))
void group_representatives(const int64_t* ids, int64_t n, int64_t* rep, hipStream_t s);
// idx[g * size + j] = perm[offs[g] + j]: row ids of G segments of one size
void segment_rows(const int64_t* perm, const int64_t* offs, int64_t G, int64_t size, int64_t* idx, hipStream_t s);
// dst row idx[j] = src row j (rows of row_bytes bytes)
void scatter_rows(int64_t row_bytes, const void* src, const int64_t* idx, void* dst, int64_t nidx, hipStream_t s);
// shuffle records: column c of a row occupies bytes [off[c], off[c] + row_bytes[c])
// of an R-byte record (off ascending, word-aligned slots when possible)
constexpr int kMaxPackCols = 16;
struct PackCols {
  int n = 0;
  int64_t row_bytes[kMaxPackCols];
  int64_t off[kMaxPackCols];
  const void* ptr[kMaxPackCols];
};
// out[j] = record of source row perm[j] (perm null: row j)
void pack_rows(const PackCols& pc, const int64_t* perm, int64_t nrows, int64_t record_bytes, void* out,
               hipStream_t s);
// column buffers pc.ptr[c] [nrows, row_bytes[c]] <- records
void unpack_rows(const PackCols& pc, const void* in, int64_t nrows, int64_t record_bytes, hipStream_t s);
// rows ordered by destination (stable): perm [n]; counts [world] rows per destination
size_t partition_workspace_bytes(int64_t n);
void partition_rows(const int64_t* dest, int64_t n, int64_t world, int64_t* perm, int64_t* counts, void* workspace,
                    size_t workspace_size, hipStream_t s);

// ------------------------------------------------------------ data movement
// dst[idx] = src[idx] over `dims`, both operands addressed by element strides
// (src strides may be 0 or negative; pointers already include the offsets).
constexpr int kMaxCopyPieces = 32;
struct CopyPieces {
  const void* src[kMaxCopyPieces];
  int64_t dst_off[kMaxCopyPieces];
  int64_t bytes[kMaxCopyPieces];
  int n = 0;
};
void batched_copy(const CopyPieces& pc, void* dst, hipStream_t s);
void strided_copy(int64_t elem_size, int rank, const int64_t* dims, const void* src,
                  const int64_t* src_strides, void* dst, const int64_t* dst_strides,
                  hipStream_t s);
// Gather rows: out[o, j, i] = params[o, idx[j], i]
void gather(int64_t elem_size, DType idt, const void* params, const void* idx, void* out,
            int64_t outer, int64_t axis_dim, int64_t nidx, int64_t inner, hipStream_t s);
void one_hot(DType dt, DType idt, const void* idx, void* out, int64_t n, int64_t depth,
             double on, double off, hipStream_t s);

// ------------------------------------------------------------ GEMM (MFMA)
// GEMM/conv epilogue activations (planner-fused unary op after the product
// and its bias); the formulas match the standalone elementwise kernels
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2, ACT_SIGMOID = 3, ACT_TANH = 4, ACT_ELU = 5,
                 ACT_SELU = 6, ACT_SOFTPLUS = 7 };

// Elementwise chain absorbed into the GEMM/conv epilogue: after bias and
// activation, v = op_k(v, x_k) for k < n, where x_k is a scalar, a per-column
// [N] vector, a per-row [M] vector or a full [batch, M, N] tensor (the
// planner's match of ops that follow the product; formulas as the
// standalone elementwise kernels)
enum EpiCode : int { EPI_ADD = 0, EPI_SUB, EPI_RSUB, EPI_MUL, EPI_DIV, EPI_RDIV, EPI_MAX, EPI_MIN, EPI_ACT, EPI_NEG,
                     EPI_SQUARE, EPI_ABS };
enum EpiOperand : int { EPO_NONE = 0, EPO_SCALAR, EPO_SCALAR_PTR, EPO_COL, EPO_ROW, EPO_FULL };
struct EpiOp {
  int code = EPI_ADD, kind = EPO_NONE, act = ACT_NONE;
  double s = 0;              // EPO_SCALAR value
  const void* p = nullptr;   // device operand (same dtype as the output)
};
constexpr int kMaxEpi = 6;
struct EpiProg {
  int n = 0;
  EpiOp op[kMaxEpi];
};

// Output column segments (horizontally fused sibling convs): columns
// [begin[s], begin[s+1]) of the product go to their own tensor ptr[s] with
// row stride ldc[s] (column begin[s] lands at ptr[s][0]); n == 0: one output C.
constexpr int kMaxOutSegs = 4;
struct OutSegs {
  int n = 0;
  int64_t begin[kMaxOutSegs + 1];
  void* ptr[kMaxOutSegs];
  int64_t ldc[kMaxOutSegs];
  int act[kMaxOutSegs];  // per-segment activation (used in place of GemmArgs::act)
};

// C[b] = op(A[b]) @ op(B[b]) (+ bias[N]) (relu); row-major, leading dims in elements.
struct GemmArgs {
  int64_t M, N, K;
  const void* A; int64_t lda; int64_t strideA;
  const void* B; int64_t ldb; int64_t strideB;
  void* C; int64_t ldc; int64_t strideC;
  bool ta, tb;
  const void* bias;  // nullable, length N
  int act;           // epilogue activation: an Act code
  int64_t batch;
  void* workspace = nullptr;  // split-K partials (gemm_workspace_bytes)
  EpiProg epi;                // absorbed elementwise chain (epi.n == 0: none)
  OutSegs seg;                // split output (seg.n == 0: C / ldc)
};
// bytes of scratch the launch needs (0 = none); allocate before the launch
size_t gemm_workspace_bytes(DType dt, const GemmArgs& g);
void gemm(DType dt, const GemmArgs& g, hipStream_t s);
// Compute mode of float32 MatMul / Conv2D: 0 exact f32 (default), 1 bf16
// operands, 2 bf16x3 (hi/lo split, ~16-bit operands); f32 accumulate in all.
// Initial value from TFA_PRECISION (f32 | bf16 | bf16x3).
void set_f32_precision(int mode);
// Force one tile of the f32 core (-1 = heuristic + autotuner); for tests/tuning.
void set_gemm_tile(int cfg);
int gemm_tile_count();
// the autotuner's picks ({20-field shape key, tile}) and the shipped defaults
// it starts from (a default is replaced only by a >= 2 % win, confirmed twice)
std::vector<std::pair<std::vector<int64_t>, int>> gemm_tune_table();
void gemm_tune_seed(const std::vector<int64_t>& key, int cfg);
void gemm_tune_reset();
std::vector<int> gemm_tile_dims(int cfg);  // {BM, BN, core (1 round-4, 2 g2)}
int f32_precision();

// ------------------------------------------------------------ conv / pool (NHWC)
struct ConvArgs {
  int64_t N, H, W, C;       // input
  int64_t KH, KW, OC;       // filter [KH, KW, C, OC]
  int64_t OH, OW;
  int64_t sh, sw, dh, dw;
  int64_t pad_t, pad_l;
  const void* x; const void* w; void* y;
  const void* bias; int act;
  void* workspace = nullptr;
  int64_t ldc = 0;  // output pixel stride in elements (0 = OC; > OC writes a channel slice)
  EpiProg epi;      // absorbed elementwise chain over the [N*OH*OW, OC] output
  OutSegs seg;      // sibling convs fused along OC: per-sibling outputs (seg.n == 0: y / ldc)
  // Winograd filter (conv_wino_filter layout) when the planner made one:
  // 3x3 / 1x7 / 7x1 stride-1 convs then run conv_wino.hip unless TFA_CONV_ALGO=direct
  const void* wino = nullptr;
  // planner-fused 2x2 / stride 2 VALID MaxPool after the conv (and its bias /
  // activation): y is the pooled [N, OH/2, OW/2] output (ldc as above). Only
  // where conv2d_pool2_direct says so (the F(2x2,3x3) epilogue pools its own
  // 2x2 output tiles); run_conv2d falls back to conv + pool otherwise.
  bool pool2 = false;
};
size_t conv2d_workspace_bytes(DType dt, const ConvArgs& a);
void conv2d_nhwc(DType dt, const ConvArgs& a, hipStream_t s);
bool conv2d_pool2_direct(const ConvArgs& a);
// the kernel family the calling thread's last conv2d_nhwc ran ("wino_f23",
// "implicit_gemm", "gemm_1x1", "direct", ...): step-timing labels
const char* last_conv_algo();
void set_last_conv_algo(const char* label);  // a static string
const char* last_f32_tile();  // " g2 256x64" etc.: the tile of the calling thread's last f32 GEMM / conv ("" if none)
struct PoolArgs {
  int64_t N, H, W, C, OH, OW, KH, KW, sh, sw, pad_t, pad_l;
  bool is_max;
  const void* x; void* y;
  // fused epilogue (planner: Pool -> BiasAdd -> Relu/Relu6) and output pixel
  // stride (> C: the pool writes its channel slice of a concat output)
  const void* bias = nullptr;  // [C] f32 or null
  int act = 0;                 // Act code (none / relu / relu6)
  int64_t ldc = 0;             // 0 = C
};
void pool2d_nhwc(DType dt, const PoolArgs& a, hipStream_t s);
// VALID 3x3 max pool (any stride) feeding a 1x1 / stride-1 conv (+ bias + act) in one kernel
// (conv_smallc.hip): Inception-v3 MaxPool_3a -> Conv2d_3b. The pooled tensor
// never reaches HBM. x: the pool's NHWC input; w: [C][OC]; y: [N*PH*PW][ldc].
struct PoolConvArgs {
  int64_t N, H, W, C, PH, PW, pkh, pkw, psh, psw, OC, ldc;
  const void* x; const void* w; const void* bias; void* y;
  int act = 0;
};
bool pool_conv1x1_eligible(int64_t N, int64_t H, int64_t W, int64_t C, int64_t PH, int64_t PW, int64_t OC,
                           int64_t ldc, int act);
void pool_conv1x1(const PoolConvArgs& a, hipStream_t s);
// Winograd paths (conv_wino.hip): the planner's shape test (0 none, 1
// F(2x2,3x3), 2 F(2,7) along W (1x7), 3 F(2,7) along H (7x1)), padded filter
// width, runtime switch (TFA_CONV_ALGO=direct turns it off) and forced
// kernel variant (-1 auto; >= 0 also runs OC <= 32; 3 one item per block)
int conv_wino_kind(int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t dh, int64_t dw, int64_t C, int64_t OC);
int64_t conv_wino_ocp(int64_t OC);
int64_t conv_wino_filter_elems(int kind, int64_t C, int64_t OC);
// host: HWIO f32 filter -> the transformed filter (fp64 transform, rounded once)
void conv_wino_filter(int kind, const float* w, int64_t C, int64_t OC, float* u);
void set_conv_wino(int on);
bool conv_wino_enabled();
void set_wino_tile(int v);
void set_wino_bn(int bn);  // F(2x2,3x3) oc block: 0 auto, 32 or 64
void set_wino_5x5(int on);  // F(4,5) for 5x5 convs (opt-in; plans made after the call)
// image resize, NHWC. mode: 0 legacy (src = dst*scale), 1 align_corners, 2 half_pixel_centers
struct ResizeArgs {
  int64_t N, H, W, C, OH, OW;
  float sh, sw;  // in/out scale per axis
  int mode;
  const void* x; void* y;
};
void resize_bilinear(DType dt, const ResizeArgs& a, hipStream_t s);  // output f32
void resize_nearest(int64_t elem_size, const ResizeArgs& a, hipStream_t s);
// batched ragged image pre-stage: n uint8 HWC images of their own sizes (byte
// offsets offs[n], (H, W) pairs hw[2n]) -> f32 [n, h, w, C]: bilinear resize
// to OH x OW (mode 0 default, 1 align_corners, 2 half_pixel_centers), crop at
// (oy, ox), then up to 4 elementwise steps (0 add, 1 sub, 2 mul, 3 div; a
// scalar or per-channel constant). rp (optional, int32 [n][4]): each row's
// own OH, OW, oy, ox instead of the shared ones.
struct RaggedPrepArgs {
  int64_t n = 0;
  int C = 3, OH = 0, OW = 0, oy = 0, ox = 0, h = 0, w = 0, mode = 0;
  int nops = 0;
  int op_kind[4] = {0, 0, 0, 0}, op_chan[4] = {0, 0, 0, 0};
  float op_val[4][4] = {};
  const uint8_t* x = nullptr;
  const int64_t* offs = nullptr;
  const int32_t* hw = nullptr;
  const int32_t* rp = nullptr;
  float* y = nullptr;
};
void ragged_image_prep(const RaggedPrepArgs& a, hipStream_t s);
// ------------------------------------------------------------ wider op set (extra.hip)
// Pad / PadV2 (mode 0, constant = cbits reinterpreted as the element) and
// MirrorPad (mode 1 REFLECT, 2 SYMMETRIC); in_strides in elements
struct PadArgs {
  int rank = 0, mode = 0;
  int64_t out_dims[kMaxRank], in_dims[kMaxRank], in_strides[kMaxRank], before[kMaxRank];
};
void pad_nd(int64_t elem_size, const PadArgs& a, const void* x, void* y, uint64_t cbits, hipStream_t s);
// cumulative sum / product along the middle dim of [outer, n, inner]
void scan(bool prod, DType dt, const void* x, void* y, int64_t outer, int64_t n, int64_t inner, bool exclusive,
          bool reverse, hipStream_t s);
void leaky_relu(DType dt, const void* x, void* y, int64_t n, double alpha, hipStream_t s);
struct DepthwiseArgs {
  int64_t N, H, W, C, M, KH, KW, OH, OW, sh, sw, dh, dw, pad_t, pad_l;
  const void* x; const void* w; void* y;
};
void depthwise_conv2d_nhwc(const DepthwiseArgs& a, hipStream_t s);  // f32
void lrn(DType dt, const void* x, void* y, int64_t n, int64_t C, int radius, double bias, double alpha, double beta,
         hipStream_t s);
struct GatherNdArgs {
  int K = 0;
  int64_t dims[kMaxRank], strides[kMaxRank];  // strides in units of `inner` slices
};
void gather_nd(int64_t elem_size, DType idt, const void* params, const void* idx, void* out, int64_t nidx,
               int64_t inner, const GatherNdArgs& a, hipStream_t s);
struct WhereArgs {
  int rank = 0;
  int64_t dims[kMaxRank];
};
// pos = inclusive prefix count of mask (int64); where_coords writes [count, rank]
void mask_prefix(const uint8_t* mask, int64_t* pos, int64_t n, hipStream_t s);
void where_coords(const uint8_t* mask, const int64_t* pos, int64_t* out, int64_t n, const WhereArgs& a,
                  hipStream_t s);

// y = x * scale[c] + shift[c] (+relu), channel = last dim
void channel_affine(DType dt, const void* x, const void* scale, const void* shift, void* y,
                    int64_t n, int64_t C, int act, hipStream_t s);

}  // namespace k
}  // namespace tfa
