// f32 MFMA GEMM + implicit-GEMM Conv2D for gfx950 (CDNA4).
//
// v_mfma_f32_32x32x2_f32 (exact f32: gfx950 has no xf32). One kernel
// template (gemm_f32_core.h, instantiated per A loader in gemm_f32_*.hip)
// over the block tile BMxBN (4, 8 or 16 waves arranged WMxWN, each wave
// owning (BM/WM)x(BN/WN) as 32x32 MFMA tiles) so the tile can follow the
// problem: 256x256 / 128x256 / 256x128 for big GEMMs, 128x192 / 64x64 /
// 128x32 and friends for narrow conv layers, split-K for grids that cannot
// fill 256 CUs. This file holds the tile table, the plans, the autotuner and
// the entry points.
//
//  * k-major LDS images (As[k][m], Bs[k][n]): every MFMA operand read is 32
//    consecutive floats per half-wave (conflict-free ds_read_b32);
//  * two LDS stages; the next K tile's global loads are issued during the
//    current tile's MFMAs (register-staged pipeline, one barrier per tile),
//    with every memory op interleaved between MFMAs (sched_group_barrier);
//  * bias + ReLU/ReLU6 fused into the epilogue (or into the split-K reducer);
//  * XCD-aware bijective block->tile remap: blocks sharing an A row panel
//    run on one XCD and share its L2.
// Conv2D (NHWC, filter HWIO) uses the same core with an im2col-on-the-fly A
// loader: A[m = (n,oh,ow)][k = (kh,kw,c)], B = filter viewed as [KH*KW*C, OC];
// 1x1 stride-1 convs are plain GEMMs over x viewed as [N*H*W, C].
#include <array>
#include <atomic>
#include <cmath>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>

#include "gemm_f32_core.h"
#include "gemm_g2_core.h"
#include "gemm_internal.h"
#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

using namespace f32core;

// split-K combine: fixed summation order over the splits (deterministic)
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ ws, GemmArgs g, int splits) {
  const int64_t M = g.M, N = g.N;
  const int64_t total = g.batch * M * N;
  const float* bias = static_cast<const float*>(g.bias);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[z * total + i];
    const int64_t col = i % N;
    const int64_t row = (i / N) % M;
    const int64_t b = i / (M * N);
    if (bias) s += bias[col];
    float* cbase;
    int64_t cld;
    int cact;
    out_col(g, static_cast<float*>(g.C) + b * g.strideC, col, cbase, cld, cact);
    cbase[row * cld] = epi_apply(g.epi, act_apply(s, cact), row, col, N, b * M * N);
  }
}

// ------------------------------------------------------------------ tile choice

// measured (scripts/gemm_bench.py, scripts/bigtile_lab.hip): 128x256 and BK=32 variants were slower on every
// shape; 256x128 (wave tile 128x64) pays only with the interleaved schedule (+8-12% on big GEMMs) and
// loses on grids of a few hundred blocks
// {BM, BN}; the N-widths 96/160/192 fit Inception-style channel counts without
// padding a 128-wide tile (a 128 tile on N=96 computes 25% zeros)
// 13-15 are 8-wave blocks (512 threads). Measured (scripts/tile_ab.sh,
// profiles/r3_tiles/): the 8-wave 256x128 wins 4096^3 (137.5 TF vs 133.6 for
// 128x128) and ties the headline 2.5Mx512x512; 256x96 (8x1) and 128x128 (2x4)
// win some Inception convs. 256x192, a BK=32 256x128 and BK=32 128x64 /
// 128x32 (one whole C=32 filter tap per k tile) never won.
// 16-18 are 8-wave versions of narrow conv tiles: 128x192 as 4x2 waves
// (each 32x96, the wave tile of 64x192), 256x64 as 8x1 (each 32x64) and
// 128x64 as 4x2 (each 32x32, the wave tile of 64x64): the block's A and B
// tiles are shared by twice the waves (less global and LDS traffic per FLOP)
// at the same wave tile. 256x160 as 8x1 never won (profiles/r4_tiles/).
// 19-20 are 8-wave 128x256 (4x2 waves of 32x128) and 256x256 (4x2 waves of
// 64x128, 1 block per CU): 4096^3 137.5 -> 140.9 TF, 8192^3 140.8 -> 142.2 TF,
// 2.5M x 512 x 512 134.8 -> 135.6 TF; a 2x4 128x256 never beat them.
// 21 is 256x256 as 16 waves (4x4 waves of 64x64, 1024 threads, four waves
// per SIMD in one block): 4096^3 141.2 TF, 8192^3 142.6 TF.
// 22-31 are the g2 core (gemm_g2_core.h: one wave per SIMD or two-block
// tiles, LDS-DMA staging, k-octet b128 fragments), kG2Tiles in order; used where its loaders apply
// (k-contiguous A or the conv im2col with C % 4 == 0, 16-byte aligned rows).
constexpr int kFirstG2 = 22;
constexpr int kNumTiles = kFirstG2 + g2::kNumG2Tiles;
constexpr int kTiles[kNumTiles][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}, {128, 32},
                                      {128, 96}, {128, 192}, {128, 160}, {64, 192}, {256, 128},
                                      {256, 64}, {256, 32}, {256, 96}, {256, 128}, {256, 96},
                                      {128, 128}, {128, 192}, {256, 64}, {128, 64}, {128, 256},
                                      {256, 256}, {256, 256},
                                      // g2
                                      {256, 256}, {256, 192}, {256, 128}, {256, 64}, {128, 128}, {128, 64},
                                      {128, 192}, {256, 96}, {128, 160}, {192, 192}, {128, 224}};
static_assert(g2::kG2Tiles[0][0] == 256 && g2::kG2Tiles[0][1] == 256 && g2::kG2Tiles[5][1] == 64 &&
                  g2::kG2Tiles[6][1] == 192 && g2::kG2Tiles[7][1] == 96 && g2::kG2Tiles[8][1] == 160 &&
                  g2::kG2Tiles[9][0] == 192 && g2::kG2Tiles[10][1] == 224,
              "kTiles' g2 rows mirror kG2Tiles");

// the g2 core's loaders: k-contiguous A (or the vec conv loader), 16-byte
// aligned operand rows, whole 4-column quads of B [K][N]
bool g2_ok(const GemmArgs& g, int al, bool vec) {
  static const bool off = [] {
    const char* e = std::getenv("TFA_GEMM_G2");
    return e && std::atoi(e) == 0;
  }();
  if (off || !vec || (al != A_KCONTIG && al != A_CONV)) return false;
  if (!g.tb && g.N % 4 != 0) return false;
  // per-lane source offsets are 32-bit bytes within a 256-row block
  constexpr int64_t kMaxLd = (int64_t(1) << 32) / (256 * 4) - 64;
  if ((al == A_KCONTIG && g.lda > kMaxLd) || g.ldb > kMaxLd) return false;
  return g.K % 4 == 0;
}

int64_t tile_blocks(int c, int64_t M, int64_t N, int64_t batch) {
  return ((M + kTiles[c][0] - 1) / kTiles[c][0]) * ((N + kTiles[c][1] - 1) / kTiles[c][1]) * batch;
}

// the launch plan of tile `cfg`: split K when the grid is under one block per CU
F32Plan plan_for(int cfg, int64_t M, int64_t N, int64_t K, int64_t batch) {
  F32Plan p{cfg, kTiles[cfg][0], kTiles[cfg][1], 1, K};
  const int64_t nb = tile_blocks(cfg, M, N, batch);
  if (nb < 256 && K >= 256) {  // each split >= 128 deep
    int64_t s = std::min<int64_t>((512 + nb - 1) / nb, K / 128);
    s = std::max<int64_t>(1, std::min<int64_t>(s, 16));
    int64_t kps = ((K + s - 1) / s + kSplitAlign - 1) / kSplitAlign * kSplitAlign;
    p.splits = (int)((K + kps - 1) / kps);
    p.k_per_split = kps;
  }
  return p;
}

// forced f32 tile (-1 = heuristic + autotuner): TFA_GEMM_TILE or set_gemm_tile()
std::atomic<int>& forced_tile() {
  static std::atomic<int> v([] {
    const char* e = std::getenv("TFA_GEMM_TILE");
    const int t = e ? std::atoi(e) : -1;
    return t >= 0 && t < kNumTiles ? t : -1;
  }());
  return v;
}
int tile_env() { return forced_tile().load(); }

// Heuristic plan (also the fallback of the autotuner and what sizes the split-K workspace)
F32Plan plan_f32(int64_t M, int64_t N, int64_t K, int64_t batch, bool use_forced = true) {
  // narrow N picks a narrow tile (a 128-wide tile on N=32 wastes 3/4 of the MFMAs)
  int cfg = N <= 32 ? 4 : (N <= 64 ? 1 : 0);
  // big GEMMs: 256x64 with the 4 waves stacked along M (each 64x64, B fragments shared);
  // measured best on 2.5Mx512x512, 262kx512x512, 4096^3 and 8192x1024^2 (scripts/bigtile_lab.hip)
  if (cfg == 0 && tile_blocks(10, M, N, batch) >= 512) cfg = 10;
  // too few blocks to fill 256 CUs twice: shrink the tile
  if (tile_blocks(cfg, M, N, batch) < 512) {
    if (cfg == 0) cfg = N > 96 ? 2 : 3;
    else if (cfg == 1) cfg = 3;
  }
  if (use_forced && tile_env() >= 0) cfg = tile_env();  // tuning override
  return plan_for(cfg, M, N, K, batch);
}

void launch_plan(const F32Plan& p, const GemmArgs& g, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
  if (p.cfg >= kFirstG2) {
    TFA_CHECK(g2_ok(g, al, vec), "gemm: g2 tile on an operand layout it does not load");
    F32Plan q = p;
    q.cfg -= kFirstG2;
    if (al == A_CONV) g2::launch_conv(q, g, cg, s);
    else g2::launch_kc(q, g, s);
    return;
  }
  if (al == A_CONV) launch_conv(p, g, vec, cg, s);
  else if (al == A_KCONTIG && !g.tb) launch_kcontig_b(p, g, vec, s);
  else if (al == A_KCONTIG) launch_kcontig_bt(p, g, vec, s);
  else if (!g.tb) launch_mcontig_b(p, g, vec, s);
  else launch_mcontig_bt(p, g, vec, s);
}

// ---- tile autotuner. The best tile depends on the grid the shape makes (an
// Inception 12x12 conv runs 35% faster on 64x64 tiles than on 128x128, the
// 10M-row headline GEMM is fastest on 128x128), so the first launch of a new
// (shape, loader) times the single-pass tiles on the caller's stream and keeps
// the fastest. Split-K shapes keep the heuristic plan (the summation order, and
// so the result bits, never depend on a timing). Never during stream capture.
// TFA_GEMM_AUTOTUNE=0 disables it; TFA_GEMM_TILE=<cfg> forces a tile.
using TuneKey = std::array<int64_t, 20>;
std::mutex& tune_mu() {
  static std::mutex m;
  return m;
}
std::map<TuneKey, int>& tune_cache() {
  static std::map<TuneKey, int> c;
  return c;
}
// the shipped gfx950 defaults (tensorframes_amd/tiles/gfx950.json, seeded at
// import): a shape with a default keeps it unless a challenger wins by >= 2 %
// in two independent timing passes, so boxes agree on the tile (and the
// bits) instead of following timing noise
std::map<TuneKey, int>& tune_defaults() {
  static std::map<TuneKey, int> d;
  return d;
}
bool autotune_on() {
  static const bool v = [] {
    const char* e = std::getenv("TFA_GEMM_AUTOTUNE");
    return !(e && std::atoi(e) == 0);
  }();
  return v && tile_env() < 0;
}

F32Plan tuned_plan(const F32Plan& heur, const GemmArgs& g0, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
  GemmArgs g = g0;
  g.workspace = nullptr;  // single-pass candidates only (a workspace would select the split-K epilogue)
  const TuneKey key{g.M, g.N, g.K, g.batch, al, g.tb, vec, cg.H, cg.W, cg.C, cg.KW, cg.OH, cg.OW,
                    cg.sh, cg.sw, cg.dh, cg.dw, cg.pt, cg.pl, (g.ldc == g.N) + 2 * g.seg.n};
  {
    std::lock_guard<std::mutex> lk(tune_mu());
    auto it = tune_cache().find(key);
    if (it != tune_cache().end()) return plan_for(it->second, g.M, g.N, g.K, g.batch);
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return heur;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return heur;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return heur;
  }
  // Three rounds over the candidates (interleaved, so clock drift hits every
  // tile alike); a candidate's time is its best round, each round >= ~1 ms of
  // launches (a 3-launch round of a 0.3 ms conv was noisy enough to keep a
  // tile 3-5 % off the best; profiles/r3_tiles/)
  int reps = 3;
  {
    launch_plan(heur, g, al, vec, cg, s);  // warm
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 3; ++r) launch_plan(heur, g, al, vec, cg, s);
    (void)hipEventRecord(e1, s);
    float ms = 0.f;
    if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f)
      reps = std::max(3, std::min(16, (int)std::ceil(1.0f / (ms / 3))));
  }
  int dflt = -1;
  {
    std::lock_guard<std::mutex> lk(tune_mu());
    auto it = tune_defaults().find(key);
    if (it != tune_defaults().end() && it->second >= 0 && it->second < kNumTiles &&
        plan_for(it->second, g.M, g.N, g.K, g.batch).splits == 1 && (it->second < kFirstG2 || g2_ok(g, al, vec)))
      dflt = it->second;
  }
  const int base = dflt >= 0 ? dflt : heur.cfg;
  // times every eligible candidate (or only `only`, >= 0) `rounds` times, interleaved
  auto time_tiles = [&](float* cand_ms, int only_a, int only_b) {
    for (int c = 0; c < kNumTiles; ++c) cand_ms[c] = 1e30f;
    for (int round = 0; round < 3; ++round) {
      for (int c = 0; c < kNumTiles; ++c) {
        if (only_a >= 0 && c != only_a && c != only_b) continue;
        const F32Plan q = plan_for(c, g.M, g.N, g.K, g.batch);
        if (q.splits != 1) continue;
        if (c >= kFirstG2 && !g2_ok(g, al, vec)) continue;
        if (c != base && kTiles[c][1] >= 2 * g.N && kTiles[c][1] > 32) continue;  // mostly-padding tile
        if (round == 0) launch_plan(q, g, al, vec, cg, s);  // warm
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) launch_plan(q, g, al, vec, cg, s);
        (void)hipEventRecord(e1, s);
        float ms = 0.f;
        if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) continue;
        cand_ms[c] = std::min(cand_ms[c], ms / reps);
      }
    }
  };
  float cand_ms[kNumTiles];
  time_tiles(cand_ms, -1, -1);
  int best = base;
  for (int c = 0; c < kNumTiles; ++c)
    if (cand_ms[c] < cand_ms[best]) best = c;
  bool replaced = false;
  if (dflt >= 0 && best != dflt) {
    // a challenger to the shipped default: >= 2 % faster, and again in a
    // second, independent pass over the two
    bool keep = !(cand_ms[best] <= 0.98f * cand_ms[dflt]);
    if (!keep) {
      float again[kNumTiles];
      time_tiles(again, dflt, best);
      keep = !(again[best] <= 0.98f * again[dflt]);
    }
    replaced = !keep;
    if (keep) best = dflt;
  }
  static const bool log = std::getenv("TFA_GEMM_TUNE_LOG") != nullptr;
  if (log) {
    std::fprintf(stderr, "[gemm tune] M=%lld N=%lld K=%lld al=%d conv=%dx%dx%d heur=%d default=%d%s best=%d |",
                 (long long)g.M, (long long)g.N, (long long)g.K, al, cg.H, cg.W, cg.C, heur.cfg, dflt,
                 replaced ? " (replaced)" : "", best);
    for (int c = 0; c < kNumTiles; ++c)
      if (cand_ms[c] < 1e29f) std::fprintf(stderr, " %d:%.4f", c, cand_ms[c]);
    std::fprintf(stderr, "\n");
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  TFA_LAUNCH_CHECK("gemm autotune");
  {
    std::lock_guard<std::mutex> lk(tune_mu());
    tune_cache()[key] = best;
  }
  return plan_for(best, g.M, g.N, g.K, g.batch);
}

namespace {
thread_local char t_tile_label[48] = "";  // the tile the calling thread's last run_f32 launched
}

void run_f32(const GemmArgs& g0, int al, bool vec, const ConvGeom& cg, hipStream_t s) {
  F32Plan p = plan_f32(g0.M, g0.N, g0.K, g0.batch);
  if (p.cfg >= kFirstG2 && !g2_ok(g0, al, vec))  // a forced g2 tile on a layout it does not load
    p = plan_f32(g0.M, g0.N, g0.K, g0.batch, false);
  if (p.splits == 1 && autotune_on()) p = tuned_plan(p, g0, al, vec, cg, s);
  GemmArgs g = g0;
  if (p.splits > 1) {
    TFA_CHECK(g0.workspace != nullptr, "gemm: split-K needs a workspace (gemm_workspace_bytes)");
  } else {
    g.workspace = nullptr;
  }
  launch_plan(p, g, al, vec, cg, s);
  std::snprintf(t_tile_label, sizeof(t_tile_label), " %s %dx%d%s", p.cfg >= kFirstG2 ? "g2" : "r4", kTiles[p.cfg][0],
                kTiles[p.cfg][1], p.splits > 1 ? " split-K" : "");
  if (p.splits > 1) {
    int64_t total = g.batch * g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce, dim3(ew_grid(total)), dim3(256), 0, s, static_cast<const float*>(g.workspace), g,
                       p.splits);
  }
}

size_t f32_ws_bytes(int64_t M, int64_t N, int64_t K, int64_t batch) {
  F32Plan p = plan_f32(M, N, K, batch);
  return p.splits > 1 ? static_cast<size_t>(p.splits) * batch * M * N * sizeof(float) : 0;
}

bool conv_is_pointwise(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.sh == 1 && a.sw == 1 && a.pad_t == 0 && a.pad_l == 0 &&
         a.OH == a.H && a.OW == a.W;
}

std::atomic<int>& precision_state() {
  static std::atomic<int> mode([] {
    const char* e = std::getenv("TFA_PRECISION");
    if (!e) return 0;
    if (!std::strcmp(e, "bf16")) return 1;
    if (!std::strcmp(e, "bf16x3")) return 2;
    return 0;
  }());
  return mode;
}

// bf16 paths: batch 1, 16-byte A rows (K % 4 / C % 4), no transposed A
bool bf16_candidate(const GemmArgs& g) {
  return f32_precision() != 0 && g.batch == 1 && !g.ta && g.lda % 4 == 0 && g.K % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(g.A) & 15) == 0;
}

GemmArgs conv_as_gemm(const ConvArgs& a) {
  GemmArgs g{};
  g.M = a.N * a.OH * a.OW;
  g.N = a.OC;
  g.K = a.KH * a.KW * a.C;
  g.A = a.x; g.lda = a.C; g.strideA = 0;
  g.B = a.w; g.ldb = a.OC; g.strideB = 0;
  g.C = a.y; g.ldc = a.ldc > 0 ? a.ldc : a.OC; g.strideC = 0;
  g.ta = false; g.tb = false;
  g.bias = a.bias;
  g.act = a.act;
  g.batch = 1;
  g.workspace = a.workspace;
  g.epi = a.epi;
  g.seg = a.seg;
  return g;
}

}  // namespace

void set_gemm_tile(int cfg) {
  TFA_CHECK(cfg >= -1 && cfg < kNumTiles, "gemm tile must be -1 (auto) or 0..", kNumTiles - 1);
  forced_tile().store(cfg);
}
int gemm_tile_count() { return kNumTiles; }

std::vector<std::pair<std::vector<int64_t>, int>> gemm_tune_table() {
  std::lock_guard<std::mutex> lk(tune_mu());
  std::vector<std::pair<std::vector<int64_t>, int>> v;
  for (const auto& kv : tune_cache()) v.emplace_back(std::vector<int64_t>(kv.first.begin(), kv.first.end()), kv.second);
  return v;
}

void gemm_tune_seed(const std::vector<int64_t>& key, int cfg) {
  TFA_CHECK(key.size() == std::tuple_size<TuneKey>::value, "gemm_tune_seed: key of ", key.size(), " fields");
  TFA_CHECK(cfg >= 0 && cfg < kNumTiles, "gemm_tune_seed: tile ", cfg, " out of range");
  TuneKey k;
  std::copy(key.begin(), key.end(), k.begin());
  std::lock_guard<std::mutex> lk(tune_mu());
  tune_defaults()[k] = cfg;
}

void gemm_tune_reset() {
  std::lock_guard<std::mutex> lk(tune_mu());
  tune_cache().clear();
}

std::vector<int> gemm_tile_dims(int cfg) {
  TFA_CHECK(cfg >= 0 && cfg < kNumTiles, "gemm_tile_dims: tile ", cfg, " out of range");
  return {kTiles[cfg][0], kTiles[cfg][1], cfg >= kFirstG2 ? 2 : 1};
}

void set_f32_precision(int mode) {
  TFA_CHECK(mode >= 0 && mode <= 2, "precision mode must be 0 (f32), 1 (bf16) or 2 (bf16x3)");
  precision_state().store(mode);
}
int f32_precision() { return precision_state().load(); }

size_t gemm_workspace_bytes(DType dt, const GemmArgs& g) {
  if (dt != DType::F32 || g.M <= 0 || g.N <= 0) return 0;
  if (bf16_candidate(g)) return bf16_workspace_bytes(f32_precision(), g.N, g.K);
  return f32_ws_bytes(g.M, g.N, g.K, g.batch);
}

size_t conv2d_workspace_bytes(DType dt, const ConvArgs& a) {
  if (dt != DType::F32) return 0;
  const GemmArgs g = conv_as_gemm(a);
  if (a.seg.n == 0 && bf16_candidate(g)) return bf16_workspace_bytes(f32_precision(), g.N, g.K);
  return f32_ws_bytes(g.M, g.N, g.K, 1);
}

const char* last_f32_tile() { return t_tile_label; }

void gemm(DType dt, const GemmArgs& g, hipStream_t s) {
  t_tile_label[0] = 0;
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return;
  TFA_CHECK(g.K > 0, "gemm: K must be > 0");
  TFA_CHECK(g.A && g.B && g.C, "gemm: null operand");
  if (dt == DType::F32 && bf16_candidate(g) && bf16_gemm_eligible(g, false, 0)) {
    bf16_gemm_launch(f32_precision(), g, false, Im2colGeom{}, s);
    return;
  }
  if (dt == DType::F32) {
    // 16-byte vector loads need 4-float aligned rows on the contiguous side
    bool vec = al16(g.A) && al16(g.B) && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
               (g.batch == 1 || (g.strideA % 4 == 0 && g.strideB % 4 == 0));
    if (!g.ta || g.tb) vec = vec && g.K % 4 == 0;
    run_f32(g, g.ta ? A_MCONTIG : A_KCONTIG, vec, ConvGeom{}, s);
  } else if (dt == DType::F64) {
    gemm_f64_launch(g, s);
  } else if (dt == DType::I32 || dt == DType::I64) {
    gemm_int_launch(dt, g, s);
  } else {
    TFA_CHECK(false, "gemm: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("gemm");
}

namespace {
thread_local const char* t_conv_algo = "";
thread_local std::string t_conv_label;
}
void set_last_conv_algo(const char* label) { t_conv_algo = label; }  // kernels outside conv2d_nhwc
// the family, plus the tile for the implicit-GEMM / 1x1 paths
const char* last_conv_algo() {
  t_conv_label = t_conv_algo;
  if (!std::strcmp(t_conv_algo, "implicit_gemm") || !std::strcmp(t_conv_algo, "gemm_1x1")) t_conv_label += t_tile_label;
  return t_conv_label.c_str();
}

bool conv2d_pool2_direct(const ConvArgs& a) {
  if (a.seg.n != 0 || a.OH % 2 != 0 || a.OW % 2 != 0 || a.KH != 3 || a.KW != 3) return false;
  ConvArgs b = a;
  b.pool2 = false;
  if (bf16_candidate(conv_as_gemm(b))) return false;  // the bf16 modes have no pooled epilogue
  return conv_wino_eligible(b);
}

void conv2d_nhwc(DType dt, const ConvArgs& a, hipStream_t s) {
  t_tile_label[0] = 0;
  TFA_CHECK(dt == DType::F32, "conv2d: f32 only");
  TFA_CHECK(a.N > 0 && a.OH > 0 && a.OW > 0 && a.OC > 0, "conv2d: empty output");
  TFA_CHECK(a.H < (1 << 30) && a.W < (1 << 30) && a.C < (1 << 30), "conv2d: dims too large");
  TFA_CHECK(a.H * a.W * a.C < (int64_t(1) << 31), "conv2d: one input image must hold < 2^31 elements");
  GemmArgs g = conv_as_gemm(a);
  if (a.pool2) {  // conv + 2x2 max pool in the Winograd epilogue
    TFA_CHECK(conv2d_pool2_direct(a), "conv2d: pooled output without a pooling kernel path");
    t_conv_algo = "wino_f23+pool2x2";
    conv_wino_launch(a, s);
    TFA_LAUNCH_CHECK("conv2d");
    return;
  }
  // the bf16 modes have no segmented epilogue: fused sibling convs stay exact f32
  if (a.seg.n == 0 && bf16_candidate(g) && bf16_gemm_eligible(g, true, a.C)) {
    Im2colGeom cg;
    cg.H = (int)a.H; cg.W = (int)a.W; cg.C = (int)a.C; cg.KW = (int)a.KW;
    cg.OH = (int)a.OH; cg.OW = (int)a.OW;
    cg.sh = (int)a.sh; cg.sw = (int)a.sw; cg.dh = (int)a.dh; cg.dw = (int)a.dw;
    cg.pt = (int)a.pad_t; cg.pl = (int)a.pad_l;
    t_conv_algo = f32_precision() == 1 ? "bf16" : "bf16x3";
    bf16_gemm_launch(f32_precision(), g, !conv_is_pointwise(a), cg, s);
    return;
  }
  if (conv_wino_eligible(a)) {  // 3x3 stride 1 with a planner-made Winograd filter
    t_conv_algo = a.KH == 3 ? "wino_f23" : a.KH == 5 ? "wino_f45" : "wino_f27";
    conv_wino_launch(a, s);
    return;
  }
  if (!conv_is_pointwise(a) && conv_smallc_eligible(a)) {  // RGB stems: filter in registers, no LDS
    t_conv_algo = "direct_smallc";
    conv_smallc_launch(a, s);
    return;
  }
  if (conv_direct_eligible(a)) {  // narrow stem convs: filter in LDS, A to registers
    t_conv_algo = "direct";
    conv_direct_launch(a, s);
    return;
  }
  if (conv_is_pointwise(a)) {  // 1x1/s1: x is already the [N*H*W, C] A matrix
    t_conv_algo = "gemm_1x1";
    bool vec = al16(a.x) && al16(a.w) && a.C % 4 == 0 && a.OC % 4 == 0;
    run_f32(g, A_KCONTIG, vec, ConvGeom{}, s);
  } else {
    ConvGeom cg;
    cg.H = (int)a.H; cg.W = (int)a.W; cg.C = (int)a.C; cg.KW = (int)a.KW;
    cg.OH = (int)a.OH; cg.OW = (int)a.OW;
    cg.sh = (int)a.sh; cg.sw = (int)a.sw; cg.dh = (int)a.dh; cg.dw = (int)a.dw;
    cg.pt = (int)a.pad_t; cg.pl = (int)a.pad_l;
    cg.fast = g.M < (int64_t(1) << 32);
    cg.fOW = make_fastdiv((uint32_t)a.OW);
    cg.fOH = make_fastdiv((uint32_t)a.OH);
    t_conv_algo = "implicit_gemm";
    bool vec = a.C % 4 == 0 && al16(a.x) && al16(a.w) && a.OC % 4 == 0;
    run_f32(g, A_CONV, vec, cg, s);
  }
  TFA_LAUNCH_CHECK("conv2d");
}

}  // namespace k
}  // namespace tfa
