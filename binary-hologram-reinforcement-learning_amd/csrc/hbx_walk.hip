// hbx_walk.hip -- device-resident greedy DBS walk on the incremental-field path.
//
// DBS.py:247-294 / DBS_1024_24.py:313-422 visit the pixels in a shuffled
// order and keep a flip iff the PSNR strictly improves.  hbx.dbs.greedy's
// host loop runs that as speculative batches (evaluate the next K candidates
// against the current base, commit the first improving one, resume after
// it) but returns to the host after every batch to find the accepted index:
// at ~50 % acceptance that is one host round trip per ~2 candidates, and the
// loop ran launch/sync-bound at ~27k candidates/s.  Here a batch is two
// launches that read their position from the walk state in device memory:
//
//   k_walk_eval    grid (bpj, K): block (x, j) streams slice x of candidate
//                  j's plane field / group intensity / target (as k_psf_eval)
//                  and writes its partial of the flip's increments
//                  (sum dI T, sum (2 I + dI) dI; f64).
//   k_walk_decide  one block: reduces every candidate's partials in fixed
//                  order, forms the PSNRs, picks the first improving candidate
//                  in visiting order and applies it: mask bit, group
//                  statistics, prev_psnr, accept log, position, stop / refresh
//                  flags, pending commit.
//   k_walk_commit  grid (bpc): if the batch accepted a flip, rewrite that
//                  plane's field and the group intensity (as k_psf_commit).
//
// (A last-block-arrives variant that folded the decision into k_walk_eval
// needed a device-scope release fence per block -- buffer_wbl2 across the
// XCDs' L2s -- and measured 67 us per 2-candidate launch against ~10 us.)
//
// Batches after the walk is done (or halted for an exact refresh) see the
// flags and return at once, so the host can enqueue many batches per
// synchronisation.  Per 1024 x 24 candidate: 16 B/px algorithmic (U_c 8, I_g 4,
// T_g 4) = 16.8 MB; per accept +24 B/px (read + write U_c and I_g).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "hbx.h"
#include "hbx_internal.hpp"

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the walk's inter-workgroup hand-off relies on gfx950's sc1 cache policy (see k_walk_step)"
#endif

namespace hbx {

namespace {

constexpr int kWalkNT = 256;

__device__ __forceinline__ int wfold(int d, int N) {
  d = (N & (N - 1)) ? ((d % N) + N) % N : (d & (N - 1));   // N = 896 is not a power of 2
  return d <= N / 2 ? d : N - d;
}

__device__ __forceinline__ void block_sum2(double& a, double& b, double (*red)[2]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) { red[w][0] = a; red[w][1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0; b = 0.0;
    for (int i = 0; i < kWalkNT / 64; ++i) { a += red[i][0]; b += red[i][1]; }
  }
}

}  // namespace

struct WalkArgs {
  uint64_t* mask;            // [CH][N][N/64]
  const float* target;       // [G][N][N]
  double* base_stats;        // [G][3]
  float2* field;             // [CH][N][N]
  float* inten;              // [G][N][N]
  const int64_t* order;      // [n_order]
  int64_t n_order;
  hbx_dbs_walk_t* w;
  int64_t* log_pos;
  double* log_psnr;
  int64_t log_cap;
  const float2* hpsf;        // [G][N][N] single-pixel fields (quadrant read)
  double* partial;           // [K][bpj][2]
  int N, P, G, K, bpj;
  float vb;
  double count, peak;
  int rel;
  int commit_only;           // fused step: apply the pending commits, evaluate nothing
};

__global__ __launch_bounds__(kWalkNT) void k_walk_eval(WalkArgs a) {
  __shared__ double red[kWalkNT / 64][2];
  hbx_dbs_walk_t* w = a.w;
  // uniform control state: written only by earlier launches' last blocks
  if (w->done || w->halt) return;
  const int64_t pos = w->pos, total = w->total < a.n_order ? w->total : a.n_order;
  const int N = a.N, P = a.P, CH = a.G * a.P;
  const size_t hw = (size_t)N * N;
  const int j = blockIdx.y;
  double sxy = 0.0, sxx = 0.0;
  if (pos + j < total) {
    const int64_t act = a.order[pos + j];
    if (act >= 0 && act < (int64_t)CH * (int64_t)hw) {
      const int ch = (int)(act / (int64_t)hw), pix = (int)(act % (int64_t)hw);
      const int g = ch / P;
      const int r = pix / N, col = pix % N;
      const uint64_t wd = a.mask[((size_t)ch * N + r) * (N / 64) + col / 64];
      const float delta = a.vb * (float)(1 - 2 * (int)((wd >> (col & 63)) & 1ull));   // before the flip
      const float invp = 1.0f / (float)P;
      const float4* U = reinterpret_cast<const float4*>(a.field + (size_t)ch * hw);
      const float4* I = reinterpret_cast<const float4*>(a.inten + (size_t)g * hw);
      const float4* T = reinterpret_cast<const float4*>(a.target + (size_t)g * hw);
      const float2* h = a.hpsf + (size_t)g * hw;
      const int nq = (int)(hw / 4);
      for (int q = blockIdx.x * kWalkNT + threadIdx.x; q < nq; q += a.bpj * kWalkNT) {
        const int y = (4 * q) / N, x0 = (4 * q) % N;
        const float4 u01 = U[2 * q], u23 = U[2 * q + 1];
        const float4 iv = I[q], tv = T[q];
        const float2* hrow = h + (size_t)wfold(y - r, N) * N;
        const float2 h0 = hrow[wfold(x0 - col, N)], h1 = hrow[wfold(x0 + 1 - col, N)];
        const float2 h2 = hrow[wfold(x0 + 2 - col, N)], h3 = hrow[wfold(x0 + 3 - col, N)];
        const float uu[8] = {u01.x, u01.y, u01.z, u01.w, u23.x, u23.y, u23.z, u23.w};
        const float hh[8] = {h0.x, h0.y, h1.x, h1.y, h2.x, h2.y, h3.x, h3.y};
        const float ii[4] = {iv.x, iv.y, iv.z, iv.w};
        const float tt[4] = {tv.x, tv.y, tv.z, tv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float dI = flip_dI(uu[2 * k], uu[2 * k + 1], hh[2 * k], hh[2 * k + 1], delta, invp);
          sxy = fma((double)dI, (double)tt[k], sxy);
          sxx = fma((double)fmaf(2.0f, ii[k], dI), (double)dI, sxx);
        }
      }
    }
  }
  block_sum2(sxy, sxx, red);
  if (threadIdx.x == 0) {
    double* o = a.partial + ((size_t)j * a.bpj + blockIdx.x) * 2;
    o[0] = sxy;
    o[1] = sxx;
  }
}

// one block: fixed-order reduction of every candidate's partials, PSNR per
// candidate, the decision (the kernel boundary after k_walk_eval makes every
// partial visible without device-scope fences in the streaming kernel)
__global__ __launch_bounds__(kWalkNT) void k_walk_decide(WalkArgs a) {
  __shared__ double red[kWalkNT / 64][2];
  __shared__ double s_ps[kWalkNT], s_sxy[kWalkNT], s_sxx[kWalkNT];
  __shared__ int64_t s_act[kWalkNT];
  hbx_dbs_walk_t* w = a.w;
  // one snapshot of the state (uniform scalar loads, one round trip)
  const hbx_dbs_walk_t ws = *w;
  if (ws.done || ws.halt) {
    if (threadIdx.x == 0) w->split_ch1 = 0;
    return;
  }
  const int64_t pos = ws.pos, total = ws.total < a.n_order ? ws.total : a.n_order;
  const int N = a.N, P = a.P, CH = a.G * a.P, G = a.G;
  const size_t hw = (size_t)N * N;
  const int64_t left = total > pos ? total - pos : 0;
  const int kv = (int)(left < (int64_t)a.K ? left : (int64_t)a.K);
  const int bpj = a.bpj;
  // the candidates' actions and the base statistics, in flight with the partials
  int64_t act = -1;
  double bs[3 * HBX_MAX_GROUPS];
  if ((int)threadIdx.x < kv) {
    act = a.order[pos + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 3 * HBX_MAX_GROUPS; ++i) bs[i] = i < 3 * G ? a.base_stats[i] : 0.0;
  }
  // fixed-order reduction, all candidates at once: tpc = 256 / pow2ceil(kv)
  // threads per candidate, lane l sums slices l, l + tpc, ... (loads issued
  // together), then a fixed xor-shuffle tree inside the lane group and, for
  // groups wider than a wave, a fixed LDS step
  int kp = 1;
  while (kp < kv) kp *= 2;
  const int tpc = kWalkNT / kp;
  const int c = threadIdx.x / tpc, l = threadIdx.x % tpc;
  double s0 = 0.0, s1 = 0.0;
  if (c < kv) {
    const double2* pp = reinterpret_cast<const double2*>(a.partial) + (size_t)c * bpj;
#pragma unroll 8
    for (int i = l; i < bpj; i += tpc) {
      const double2 v = pp[i];
      s0 += v.x;
      s1 += v.y;
    }
  }
  const int span = tpc < 64 ? tpc : 64;
  for (int off = span / 2; off >= 1; off >>= 1) {
    s0 += __shfl_xor(s0, off, 64);
    s1 += __shfl_xor(s1, off, 64);
  }
  if (tpc > 64) {   // kv <= 2: combine the group's waves in order
    if ((threadIdx.x & 63) == 0) { red[threadIdx.x / 64][0] = s0; red[threadIdx.x / 64][1] = s1; }
    __syncthreads();
    if (l == 0) {
      s0 = 0.0; s1 = 0.0;
      for (int i = 0; i < tpc / 64; ++i) { s0 += red[c * (tpc / 64) + i][0]; s1 += red[c * (tpc / 64) + i][1]; }
    }
  }
  if (l == 0 && c < kv) { s_sxy[c] = s0; s_sxx[c] = s1; }
  __syncthreads();
  if ((int)threadIdx.x < kv) {
    const int cc = threadIdx.x;
    double ps = NAN;
    if (act >= 0 && act < (int64_t)CH * (int64_t)hw) {
      const int g = (int)(act / (int64_t)hw) / P;
      // the partials are the flip's increments: candidate group sums = base + increment
      s_sxy[cc] += bs[3 * g];
      s_sxx[cc] += bs[3 * g + 1];
      double sxy2 = 0.0, sxx2 = 0.0, syy2 = 0.0;
#pragma unroll
      for (int gg = 0; gg < HBX_MAX_GROUPS; ++gg) {
        if (gg >= G) break;
        if (gg == g) { sxy2 += s_sxy[cc]; sxx2 += s_sxx[cc]; syy2 += bs[3 * gg + 2]; }
        else { sxy2 += bs[3 * gg]; sxx2 += bs[3 * gg + 1]; syy2 += bs[3 * gg + 2]; }
      }
      ps = psnr_from(sxy2, sxx2, syy2, a.count, a.rel, a.peak);
    }
    s_ps[cc] = ps;
    s_act[cc] = act;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  int acc = -1;
  for (int k = 0; k < kv; ++k)
    if (s_ps[k] > ws.prev_psnr) { acc = k; break; }   // strict (DBS_1024_24.py:355); NaN never
  hbx_dbs_walk_t nw = ws;
  nw.batches += 1;
  if (acc >= 0) {
    const int64_t aa = s_act[acc];
    const int ch = (int)(aa / (int64_t)hw), pix = (int)(aa % (int64_t)hw);
    const int g = ch / P, r = pix / N, col = pix % N;
    atomicXor(reinterpret_cast<unsigned long long*>(a.mask) + ((size_t)ch * N + r) * (N / 64) + col / 64,
              1ull << (col & 63));                                                // DBS_1024_24.py:320
    a.base_stats[3 * g] = s_sxy[acc];                                             // :358-363
    a.base_stats[3 * g + 1] = s_sxx[acc];
    const double ps = s_ps[acc];
    nw.prev_psnr = ps;
    nw.last_psnr = ps;
    const int64_t n = ws.accepted;
    if (n < a.log_cap) { a.log_pos[n] = pos + acc; a.log_psnr[n] = ps; }
    nw.accepted = n + 1;
    nw.split_ch1 = ch + 1;
    nw.split_pix = pix;
    nw.pos = pos + acc + 1;
    if (ws.stop_enabled && ps - ws.init_psnr >= ws.stop_diff) {   // DBS_ratio_0.5.py:366-372
      nw.done = 1;
      nw.stopped_early = 1;
    }
    if (ws.refresh_every > 0 && (n + 1) % ws.refresh_every == 0) nw.halt = 1;
  } else {
    if (kv > 0) nw.last_psnr = s_ps[kv - 1];
    nw.split_ch1 = 0;
    nw.pos = pos + kv;
  }
  if (nw.pos >= total) nw.done = 1;
  *w = nw;
}

// the accepted flip of the batch (mask bit already toggled): U_c += delta h,
// I_g += (|U_c'|^2 - |U_c|^2) / P
__global__ __launch_bounds__(kWalkNT) void k_walk_commit(WalkArgs a) {
  hbx_dbs_walk_t* w = a.w;
  const int ch = w->split_ch1 - 1;
  if (ch < 0) return;
  const int pix = w->split_pix;
  const int N = a.N, P = a.P;
  const size_t hw = (size_t)N * N;
  const int g = ch / P, r = pix / N, col = pix % N;
  const uint64_t wd = a.mask[((size_t)ch * N + r) * (N / 64) + col / 64];
  const float delta = a.vb * (float)(2 * (int)((wd >> (col & 63)) & 1ull) - 1);   // after the flip
  const float invp = 1.0f / (float)P;
  float4* U = reinterpret_cast<float4*>(a.field + (size_t)ch * hw);
  float4* I = reinterpret_cast<float4*>(a.inten + (size_t)g * hw);
  const float2* h = a.hpsf + (size_t)g * hw;
  const int nq = (int)(hw / 4);
  for (int q = blockIdx.x * kWalkNT + threadIdx.x; q < nq; q += gridDim.x * kWalkNT) {
    const int y = (4 * q) / N, x0 = (4 * q) % N;
    float4 u01 = U[2 * q], u23 = U[2 * q + 1];
    float4 iv = I[q];
    const float2* hrow = h + (size_t)wfold(y - r, N) * N;
    const float2 h0 = hrow[wfold(x0 - col, N)], h1 = hrow[wfold(x0 + 1 - col, N)];
    const float2 h2 = hrow[wfold(x0 + 2 - col, N)], h3 = hrow[wfold(x0 + 3 - col, N)];
    float uu[8] = {u01.x, u01.y, u01.z, u01.w, u23.x, u23.y, u23.z, u23.w};
    const float hh[8] = {h0.x, h0.y, h1.x, h1.y, h2.x, h2.y, h3.x, h3.y};
    float ii[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float ur = uu[2 * k], ui = uu[2 * k + 1];
      ii[k] += flip_dI(ur, ui, hh[2 * k], hh[2 * k + 1], delta, invp);
      uu[2 * k] = fmaf(delta, hh[2 * k], ur);
      uu[2 * k + 1] = fmaf(delta, hh[2 * k + 1], ui);
    }
    U[2 * q] = make_float4(uu[0], uu[1], uu[2], uu[3]);
    U[2 * q + 1] = make_float4(uu[4], uu[5], uu[6], uu[7]);
    I[q] = make_float4(ii[0], ii[1], ii[2], ii[3]);
  }
}

// ---------------------------------------------------------------------------
// Fused walk step (ABI v7): ONE launch per batch.
//
//   1. every block applies the previous batch's accepted flip(s) to its pixel
//      slice of the plane field(s) and group intensity(ies) (the split walk's
//      k_walk_commit), keeping the updated values in registers;
//   2. the same block evaluates the batch's K candidates on that slice against
//      the updated state: per candidate the increments sum dI T, sum (2I+dI) dI,
//      and -- TWO = true -- for every candidate pair (i, j) of one colour group
//      sum dI_i dI_j, plus, for a pair in one plane, the field cross term
//      X = 2 d_i d_j Re(h_i conj h_j) / P through sum X T, sum (2I + 2dI_i +
//      2dI_j + X) X (the exact change of sum I T / sum I^2 when BOTH flips are
//      applied: I' = I + dI_i + dI_j + X);
//   3. block partials go out as write-through (sc1) stores, each block then
//      takes a ticket on one agent-scope counter after its stores have drained;
//      the block holding the last ticket reads every partial with sc1 loads
//      (MI355X_MICROARCH.md, inter-workgroup hand-off row 1: no release fence)
//      and decides: the first candidate that strictly improves the PSNR
//      (DBS_1024_24.py:355), and -- TWO -- the first one after it that improves
//      on the state WITH it (pairwise terms), i.e. up to two accepts of the
//      serial loop per batch; the batch ends after the second accept.  It
//      toggles the mask bits, updates the group sums, the accept log and the
//      walk state, and leaves the accepted flips as the next launch's commits.
//
// A batch then costs one kernel boundary instead of three, and at acceptance
// ~0.5 visits ~3.2 candidates (K = 4, two accepts) instead of ~1.6.  Commits
// left pending when the walk is done or halted are applied by the next launch
// (it finds no candidates and only commits); the host issues one after the
// walk ends and drops them when it re-propagates exactly (the mask already
// holds every accepted flip).
constexpr int kWalkStepBlocksMax = 256;   // one block per CU (512 blocks measured slower)
constexpr int kSc1 = 16;   // buffer cache policy bit sc1 (gfx950): write-through stores, L2-fresh loads
typedef unsigned int walk_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, (int)bytes,
                                           0x00020000);
}

// fixed-order block sum of NT per-thread values into out (LDS): every thread's
// values go to LDS once, then 8 lanes per term sum 32 each and one lane per term
// the 8 (a shuffle tree per term costs ~4 us at NT = 26)
template <int NT>
__device__ __forceinline__ void block_sum_lds(const double (&v)[NT], double (*all)[kWalkNT], double (*seg)[8],
                                              double* out) {
#pragma unroll
  for (int t = 0; t < NT; ++t) all[t][threadIdx.x] = v[t];
  __syncthreads();
  if ((int)threadIdx.x < NT * 8) {
    const int t = threadIdx.x / 8, sg = threadIdx.x % 8;
    double acc = 0.0;
#pragma unroll 8
    for (int i = 0; i < kWalkNT / 8; ++i) acc += all[t][sg + 8 * i];
    seg[t][sg] = acc;
  }
  __syncthreads();
  if ((int)threadIdx.x < NT) {
    double acc = 0.0;
#pragma unroll
    for (int sg = 0; sg < 8; ++sg) acc += seg[threadIdx.x][sg];
    out[threadIdx.x] = acc;
  }
  __syncthreads();
}

struct WalkCand {
  int ch, pix, g, r, col;
  float delta;
  bool ok;
};


template <int K, bool TWO, bool PERSIST>
__global__ __launch_bounds__(kWalkNT) void k_walk_step(WalkArgs a, int* __restrict__ counter, int n_batches) {
  constexpr int NP = TWO ? K * (K - 1) / 2 : 0;
  constexpr int NT = 2 * K + 3 * NP;
  constexpr int NG = HBX_MAX_GROUPS;
  static_assert(K <= kWalkPreMax, "fused K");
  __shared__ double red_all[NT][kWalkNT];
  __shared__ double red_seg[NT][8];
  __shared__ double tot[NT];
  __shared__ double s_ps[K + NP];
  __shared__ int s_nch[2 * kWalkPreMax], s_npix[2 * kWalkPreMax];
  __shared__ uint64_t s_nwd[2 * kWalkPreMax];
  __shared__ int s_last;
  __shared__ WalkCand s_cd[K];           // the decider's candidates, indexed at run time
  hbx_dbs_walk_t* w = a.w;
  WalkPre* prep = reinterpret_cast<WalkPre*>(counter + kWalkCounters);
  // PERSIST (r03): the launch runs up to n_batches batches; between batches the grid meets at
  // a barrier -- the last-arriving block decides, writes the walk state write-through and bumps
  // the generation word the others spin on (bounded: a block that waits past kWalkSpinMax polls
  // raises the abort word and the fault / done flags, and every waiting block leaves)
  int* const gen = counter + kWalkGen;
  int* const abort_word = counter + kWalkAbort;
  __shared__ int s_gen, s_stop;
  if constexpr (PERSIST) {
    if (threadIdx.x == 0) s_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const __amdgpu_buffer_rsrc_t r_ws = wave_rsrc(w, (unsigned)sizeof(hbx_dbs_walk_t));
  const __amdgpu_buffer_rsrc_t r_pre = wave_rsrc(prep, (unsigned)sizeof(WalkPre));
  const __amdgpu_buffer_rsrc_t r_mask = wave_rsrc(a.mask, 0xffffffffu);
  const __amdgpu_buffer_rsrc_t r_bs = wave_rsrc(a.base_stats, (unsigned)(3 * HBX_MAX_GROUPS * sizeof(double)));
  // mask words and base statistics: written by the deciding block of an earlier batch, which may
  // sit on another XCD -- in a persistent launch they are read past the local L2 (sc1)
  auto ld_mask = [&](size_t word) -> uint64_t {
    if constexpr (PERSIST)
      return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r_mask, (int)(word * 8), 0, kSc1));
    else
      return a.mask[word];
  };
#pragma unroll 1
  for (int bb = 0; bb < (PERSIST ? n_batches : 1); ++bb) {
#ifdef HBX_WALK_TIMING
  uint64_t tt[12];
  tt[0] = __builtin_amdgcn_s_memrealtime();
#define HBX_TT(i) tt[i] = __builtin_amdgcn_s_memrealtime()
#else
#define HBX_TT(i)
#endif
  // the state the previous launch left, and its decider's decoded next actions: one
  // round trip, by one wave per block (48 lanes, a word each) through LDS -- when every
  // wave of the grid loaded the same two lines itself, the K = 1, 2, 4 variants
  // measured 2-27 us (mean 7.5) before the first block could start streaming
  static_assert(sizeof(hbx_dbs_walk_t) % 4 == 0 && sizeof(WalkPre) % 4 == 0, "word copies");
  constexpr int kWsWords = (int)(sizeof(hbx_dbs_walk_t) / 4), kPreWords = (int)(sizeof(WalkPre) / 4);
  static_assert(kWsWords + kPreWords <= 64, "one wave");
  __shared__ hbx_dbs_walk_t s_ws;
  __shared__ WalkPre s_pre;
  if constexpr (PERSIST) {
    __syncthreads();   // the previous batch's readers of s_ws / s_pre / s_cd are done
    if ((int)threadIdx.x < kWsWords)
      reinterpret_cast<int*>(&s_ws)[threadIdx.x] =
          __builtin_bit_cast(int, __builtin_amdgcn_raw_buffer_load_b32(r_ws, (int)threadIdx.x * 4, 0, kSc1));
    else if ((int)threadIdx.x < kWsWords + kPreWords)
      reinterpret_cast<int*>(&s_pre)[threadIdx.x - kWsWords] = __builtin_bit_cast(
          int, __builtin_amdgcn_raw_buffer_load_b32(r_pre, ((int)threadIdx.x - kWsWords) * 4, 0, kSc1));
  } else {
    if ((int)threadIdx.x < kWsWords)
      reinterpret_cast<int*>(&s_ws)[threadIdx.x] = reinterpret_cast<const int*>(w)[threadIdx.x];
    else if ((int)threadIdx.x < kWsWords + kPreWords)
      reinterpret_cast<int*>(&s_pre)[threadIdx.x - kWsWords] = reinterpret_cast<const int*>(prep)[threadIdx.x - kWsWords];
  }
  __syncthreads();
  const hbx_dbs_walk_t ws = s_ws;
  const WalkPre pre = s_pre;
  const int N = a.N, P = a.P, G = a.G, CH = G * P;
  const size_t hw = (size_t)N * N;
  const float invp = 1.0f / (float)P;
  const int cch[2] = {ws.commit_ch, ws.commit2_ch1 - 1};
  const int cpx[2] = {ws.commit_pix, ws.commit_pix2};
  const int nc = cch[0] < 0 ? 0 : (cch[1] < 0 ? 1 : 2);
  const int64_t total = ws.total < a.n_order ? ws.total : a.n_order;
  const int64_t pos = ws.pos;
  const int64_t left = (!a.commit_only && !ws.done && !ws.halt && total > pos) ? total - pos : 0;
  const int kcap = a.K < K ? a.K : K;     // a launch may run a wider variant
  const int kv = (int)(left < (int64_t)kcap ? left : (int64_t)kcap);
  if (nc == 0 && kv == 0) return;        // uniform over the grid
  HBX_TT(8);
  const bool use_pre = pre.pos == pos && pre.order == a.order && pre.n >= kv;
  // the actions that can follow this batch, order[pos + 1 .. pos + kv + 3]: loaded now
  // (only the deciding block uses them, for the next launch's WalkPre)
  const int64_t n_next = total - pos - 1;
  const int nn = (int)(n_next < (int64_t)(kv + kWalkPreMax - 1) ? (n_next > 0 ? n_next : 0) : kv + kWalkPreMax - 1);
  int64_t nact = -1;
  if ((int)threadIdx.x < nn) nact = a.order[pos + 1 + threadIdx.x];

  WalkCand cm[2], cd[K];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    cm[c].ok = c < nc;
    const int ch = cm[c].ok ? cch[c] : 0, pix = cm[c].ok ? cpx[c] : 0;
    cm[c].ch = ch; cm[c].pix = pix; cm[c].g = ch / P; cm[c].r = pix / N; cm[c].col = pix % N;
    if (use_pre) {
      cm[c].delta = pre.cdelta[c];
    } else {
      const uint64_t wd = ld_mask(((size_t)ch * N + cm[c].r) * (N / 64) + cm[c].col / 64);
      cm[c].delta = a.vb * (float)(2 * (int)((wd >> (cm[c].col & 63)) & 1ull) - 1);   // after the flip
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    int ch = 0, pix = 0;
    if (use_pre) {
      cd[j].ok = j < kv && pre.ch[j] >= 0;
      ch = cd[j].ok ? pre.ch[j] : 0;
      pix = cd[j].ok ? pre.pix[j] : 0;
    } else {
      const int64_t act = j < kv ? a.order[pos + j] : -1;
      cd[j].ok = act >= 0 && act < (int64_t)CH * (int64_t)hw;
      ch = cd[j].ok ? (int)(act / (int64_t)hw) : 0;
      pix = cd[j].ok ? (int)(act % (int64_t)hw) : 0;
    }
    cd[j].ch = ch; cd[j].pix = pix; cd[j].g = ch / P; cd[j].r = pix / N; cd[j].col = pix % N;
    if (use_pre) {
      cd[j].delta = pre.delta[j];
    } else {
      const uint64_t wd = ld_mask(((size_t)ch * N + cd[j].r) * (N / 64) + cd[j].col / 64);
      cd[j].delta = a.vb * (float)(1 - 2 * (int)((wd >> (cd[j].col & 63)) & 1ull));   // before the flip
    }
  }
  HBX_TT(1);

  double acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = 0.0;
  const int nq = (int)(hw / 4);
  // per quad: every load (pending commits, then each candidate's plane / intensity /
  // target / shifted single-pixel field) is issued before any arithmetic or store, so a
  // quad costs one memory round trip; values a commit produces replace the loaded ones
  auto ld4 = [](const float4* p) { return *p; };   // (non-temporal loads measured slower: the
  // working set of a sweep, 24 planes + 3 intensities + 3 targets = 216 MB, lives in the MALL)
  for (int q = blockIdx.x * kWalkNT + threadIdx.x; q < nq; q += gridDim.x * kWalkNT) {
    const int y = (4 * q) / N, x0 = (4 * q) % N;
    float cu[2][8], ci[2][4], chh[2][8];
    float lu[K][8], li[K][4], lt[K][4], lh[K][8];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (c >= nc) break;
      const float4* U = reinterpret_cast<const float4*>(a.field + (size_t)cm[c].ch * hw);
      const float4 u01 = ld4(U + 2 * q), u23 = ld4(U + 2 * q + 1);
      cu[c][0] = u01.x; cu[c][1] = u01.y; cu[c][2] = u01.z; cu[c][3] = u01.w;
      cu[c][4] = u23.x; cu[c][5] = u23.y; cu[c][6] = u23.z; cu[c][7] = u23.w;
      const float4 iv = ld4(reinterpret_cast<const float4*>(a.inten + (size_t)cm[c].g * hw) + q);
      ci[c][0] = iv.x; ci[c][1] = iv.y; ci[c][2] = iv.z; ci[c][3] = iv.w;
      const float2* hrow = a.hpsf + (size_t)cm[c].g * hw + (size_t)wfold(y - cm[c].r, N) * N;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float2 hv = hrow[wfold(x0 + k - cm[c].col, N)];
        chh[c][2 * k] = hv.x;
        chh[c][2 * k + 1] = hv.y;
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j >= kv || !cd[j].ok) continue;
      const float4* U = reinterpret_cast<const float4*>(a.field + (size_t)cd[j].ch * hw);
      const float4 u01 = ld4(U + 2 * q), u23 = ld4(U + 2 * q + 1);
      lu[j][0] = u01.x; lu[j][1] = u01.y; lu[j][2] = u01.z; lu[j][3] = u01.w;
      lu[j][4] = u23.x; lu[j][5] = u23.y; lu[j][6] = u23.z; lu[j][7] = u23.w;
      const float4 iv = ld4(reinterpret_cast<const float4*>(a.inten + (size_t)cd[j].g * hw) + q);
      li[j][0] = iv.x; li[j][1] = iv.y; li[j][2] = iv.z; li[j][3] = iv.w;
      const float4 tv = ld4(reinterpret_cast<const float4*>(a.target + (size_t)cd[j].g * hw) + q);
      lt[j][0] = tv.x; lt[j][1] = tv.y; lt[j][2] = tv.z; lt[j][3] = tv.w;
      const float2* hrow = a.hpsf + (size_t)cd[j].g * hw + (size_t)wfold(y - cd[j].r, N) * N;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float2 hv = hrow[wfold(x0 + k - cd[j].col, N)];
        lh[j][2 * k] = hv.x;
        lh[j][2 * k + 1] = hv.y;
      }
    }
    // commits (the second applies on top of the first when they share a plane / group)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (c >= nc) break;
      if (c == 1 && cm[1].ch == cm[0].ch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cu[1][e] = cu[0][e];
      }
      if (c == 1 && cm[1].g == cm[0].g) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ci[1][e] = ci[0][e];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float ur = cu[c][2 * k], ui = cu[c][2 * k + 1];
        ci[c][k] += flip_dI(ur, ui, chh[c][2 * k], chh[c][2 * k + 1], cm[c].delta, invp);
        cu[c][2 * k] = fmaf(cm[c].delta, chh[c][2 * k], ur);
        cu[c][2 * k + 1] = fmaf(cm[c].delta, chh[c][2 * k + 1], ui);
      }
      float4* U = reinterpret_cast<float4*>(a.field + (size_t)cm[c].ch * hw);
      U[2 * q] = make_float4(cu[c][0], cu[c][1], cu[c][2], cu[c][3]);
      U[2 * q + 1] = make_float4(cu[c][4], cu[c][5], cu[c][6], cu[c][7]);
      reinterpret_cast<float4*>(a.inten + (size_t)cm[c].g * hw)[q] = make_float4(ci[c][0], ci[c][1], ci[c][2], ci[c][3]);
    }
    float dI[K][4];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j >= kv || !cd[j].ok) {
#pragma unroll
        for (int k = 0; k < 4; ++k) dI[j][k] = 0.0f;
        continue;
      }
      // the state after the pending commits: their planes / intensities replace the loads
      if (nc > 1 && cd[j].ch == cm[1].ch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) lu[j][e] = cu[1][e];
      } else if (nc > 0 && cd[j].ch == cm[0].ch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) lu[j][e] = cu[0][e];
      }
      if (nc > 1 && cd[j].g == cm[1].g) {
#pragma unroll
        for (int e = 0; e < 4; ++e) li[j][e] = ci[1][e];
      } else if (nc > 0 && cd[j].g == cm[0].g) {
#pragma unroll
        for (int e = 0; e < 4; ++e) li[j][e] = ci[0][e];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = flip_dI(lu[j][2 * k], lu[j][2 * k + 1], lh[j][2 * k], lh[j][2 * k + 1], cd[j].delta, invp);
        dI[j][k] = d;
        acc[j] = fma((double)d, (double)lt[j][k], acc[j]);
        acc[K + j] = fma((double)fmaf(2.0f, li[j][k], d), (double)d, acc[K + j]);
      }
    }
    if constexpr (TWO) {
      int p = 0;
#pragma unroll
      for (int i = 0; i < K; ++i) {
#pragma unroll
        for (int j = i + 1; j < K; ++j, ++p) {
          if (j >= kv || !cd[i].ok || !cd[j].ok || cd[i].g != cd[j].g) continue;
          double* e = acc + 2 * K + 3 * p;
          const bool plane = cd[i].ch == cd[j].ch;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            e[0] = fma((double)dI[i][k], (double)dI[j][k], e[0]);
            if (plane) {
              const float x = 2.0f * cd[i].delta * cd[j].delta * invp *
                              fmaf(lh[i][2 * k], lh[j][2 * k], lh[i][2 * k + 1] * lh[j][2 * k + 1]);
              e[1] = fma((double)x, (double)lt[j][k], e[1]);
              const float s2 = 2.0f * (li[j][k] + dI[i][k] + dI[j][k]) + x;
              e[2] = fma((double)s2, (double)x, e[2]);
            }
          }
        }
      }
    }
  }
  HBX_TT(2);
  block_sum_lds<NT>(acc, red_all, red_seg, tot);
  HBX_TT(3);
  // partials out as write-through stores (cache policy sc1), read back by the deciding
  // block with sc1 loads (buffer ops: the loads of all partials are in flight together)
  const __amdgpu_buffer_rsrc_t rp = wave_rsrc(a.partial, (unsigned)(gridDim.x * NT * sizeof(double)));
#ifdef HBX_WALK_TIMING
  if (threadIdx.x == 0) {   // per-block start and state-load latency (debug slots after the partials)
    long long* dbg = reinterpret_cast<long long*>(a.partial + NT * gridDim.x);
    __hip_atomic_store(dbg + 2 * blockIdx.x, (long long)tt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dbg + 2 * blockIdx.x + 1, (long long)(tt[8] - tt[0]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
  // term-major ([NT][blocks]): the deciding block's lanes then read consecutive words
  if ((int)threadIdx.x < NT)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(walk_u32x2, tot[threadIdx.x]), rp,
                                          (int)((threadIdx.x * gridDim.x + blockIdx.x) * sizeof(double)), 0, kSc1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // Memory ordering of this hand-off: the partials go out as sc1
    // (write-through) buffer stores and s_waitcnt vmcnt(0) above retires them before the
    // ticket is taken; the deciding block reads them with sc1 loads, which miss its own
    // XCD's L2.  So the RELAXED agent-scope ticket suffices on gfx950's cache policy --
    // not under the language memory model, which would need a release / acquire pair.
    // An agent-scope release here is a buffer_wbl2 of every XCD's L2 and measured 67 us
    // per launch, so the ordering is pinned to the ISA instead: this file
    // builds for gfx950 only (the #error at the top), and every walk test checks the accept
    // sequence against the float64 oracle.  One arrival counter (a two-level counter
    // sharded by XCD measured 30.6 vs 29.4 us per batch).
    s_last = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) {
    if constexpr (!PERSIST) {
      return;
    } else {
      // wait for the deciding block's generation bump (bounded; see above)
      if (threadIdx.x == 0) {
        int stop = 0;
        unsigned polls = 0;
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == s_gen) {
          if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { stop = 1; break; }
          if (++polls > kWalkSpinMax) {
            __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the walk state is unreliable from here: fault + done stop the caller
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 1), r_ws,
                                                  (int)offsetof(hbx_dbs_walk_t, fault), 0, kSc1);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 1), r_ws,
                                                  (int)offsetof(hbx_dbs_walk_t, done), 0, kSc1);
            stop = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
        s_stop = stop;
        s_gen = s_gen + 1;
      }
      __syncthreads();
      if (s_stop) return;
      continue;
    }
  }
  HBX_TT(4);

  // ---- the last block: every partial (fixed order), the PSNRs, the decision ----
  const int tid = threadIdx.x;
  // issued together: the next actions' mask words, the base statistics, every partial
  int nch = -1, npix = 0;
  uint64_t nwd = 0;
  if (tid < nn && nact >= 0 && nact < (int64_t)CH * (int64_t)hw) {
    nch = (int)(nact / (int64_t)hw);
    npix = (int)(nact % (int64_t)hw);
    nwd = ld_mask(((size_t)nch * N + npix / N) * (N / 64) + (npix % N) / 64);
  }
  double bs[3 * NG];
#pragma unroll
  for (int i = 0; i < 3 * NG; ++i) {
    if constexpr (PERSIST)
      bs[i] = i < 3 * G ? __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r_bs, i * 8, 0, kSc1)) : 0.0;
    else
      bs[i] = i < 3 * G ? a.base_stats[i] : 0.0;
  }
  double v[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) v[t] = 0.0;
  for (int b = tid; b < (int)gridDim.x; b += kWalkNT) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
      v[t] += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                             rp, (int)((t * gridDim.x + b) * sizeof(double)), 0, kSc1));
  }
  if (tid < nn) {
    s_nch[tid] = nch;
    s_npix[tid] = npix;
    s_nwd[tid] = nwd;
  }
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) s_cd[j] = cd[j];
  }
  HBX_TT(5);
  block_sum_lds<NT>(v, red_all, red_seg, tot);
  HBX_TT(6);
  // the PSNRs: lane j < K = candidate j on the base, lane K + p = pair p = (i, j), i < j,
  // both flips on the base (the state after accepting i, then j) -- the summation order
  // of a serial pass, so the decision is the same
  auto psnr_of = [&](const double (&st)[3 * NG]) {
    double sxy = 0.0, sxx = 0.0, syy = 0.0;
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) {
      if (gg >= G) break;
      sxy += st[3 * gg]; sxx += st[3 * gg + 1]; syy += st[3 * gg + 2];
    }
    return psnr_from(sxy, sxx, syy, a.count, a.rel, a.peak);
  };
  // adds candidate i's increments (and, for the second of a pair in the same group, the
  // pair terms) to st in place
  auto add_cand = [&](double (&st)[3 * NG], int i) {
    const int g = s_cd[i].g;
    const double dxy = tot[i], dxx = tot[K + i];
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) {     // unconditional adds (+ 0 elsewhere): no indexed
      st[3 * gg] += gg == g ? dxy : 0.0;   // access, which would put st in scratch
      st[3 * gg + 1] += gg == g ? dxx : 0.0;
    }
  };
  auto add_pair = [&](double (&st)[3 * NG], int i, int j) {
    const int g = s_cd[j].g;
    add_cand(st, j);
    if (g == s_cd[i].g) {
      const int p = i * (2 * K - i - 1) / 2 + (j - i - 1);   // index of (i < j), row-major
      const double dxy = tot[2 * K + 3 * p + 1], dxx = 2.0 * tot[2 * K + 3 * p] + tot[2 * K + 3 * p + 2];
#pragma unroll
      for (int gg = 0; gg < NG; ++gg) {
        st[3 * gg] += gg == g ? dxy : 0.0;
        st[3 * gg + 1] += gg == g ? dxx : 0.0;
      }
    }
  };
  if (tid < K + NP) {
    int i = tid, j = -1;
    if (tid >= K) {                      // pair index -> (i, j)
      int p = tid - K;
      i = 0;
      while (p >= K - 1 - i) { p -= K - 1 - i; ++i; }
      j = i + 1 + p;
    }
    double ps = NAN;
    if (i < kv && s_cd[i].ok && (j < 0 || (j < kv && s_cd[j].ok))) {
      double st[3 * NG];
#pragma unroll
      for (int e = 0; e < 3 * NG; ++e) st[e] = bs[e];
      add_cand(st, i);
      if (j >= 0) add_pair(st, i, j);
      ps = psnr_of(st);
    }
    s_ps[tid] = ps;
  }
  __syncthreads();
  if (tid == 0) {
  HBX_TT(9);
  HBX_TT(10);
  for (int i = 0; i < kWalkTickets; ++i)
    __hip_atomic_store(counter + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  hbx_dbs_walk_t nw = ws;
  nw.commit_ch = -1;
  nw.commit_pix = 0;
  nw.commit2_ch1 = 0;
  nw.commit_pix2 = 0;
  int64_t new_pos = pos;
  int acc_j[2] = {-1, -1};
  if (kv > 0) {
    nw.batches += 1;
    double prev = ws.prev_psnr, last = NAN;
    int64_t n_acc = ws.accepted;
    new_pos = pos + kv;
    bool stop = false;
    double acc_ps[2] = {NAN, NAN};
    int a0 = -1;
    for (int j = 0; j < kv; ++j) {         // first accept against the base
      last = s_ps[j];
      if (last > prev) { a0 = j; break; }  // strict (DBS_1024_24.py:355); NaN never
    }
    if (a0 >= 0) {
      double fin[3 * NG];
#pragma unroll
      for (int e = 0; e < 3 * NG; ++e) fin[e] = bs[e];
      add_cand(fin, a0);
      prev = last;
      acc_j[0] = a0;
      acc_ps[0] = last;
      new_pos = pos + a0 + 1;
      const bool halt0 = ws.refresh_every > 0 && (n_acc + 1) % ws.refresh_every == 0;
      const bool stop0 = ws.stop_enabled && prev - ws.init_psnr >= ws.stop_diff;   // DBS_ratio_0.5.py:366-372
      n_acc += 1;
      stop = stop0;
      if (halt0) nw.halt = 1;
      if constexpr (TWO) {
        if (!halt0 && !stop0) {            // second accept: candidates after a0 on the state with a0
          const WalkCand c0 = s_cd[a0];
          new_pos = pos + kv;
          for (int j = a0 + 1; j < kv; ++j) {
            const WalkCand cj = s_cd[j];
            if (cj.ok && cj.ch == c0.ch && cj.pix == c0.pix) { new_pos = pos + j; break; }
            last = s_ps[K + a0 * (2 * K - a0 - 1) / 2 + (j - a0 - 1)];
            if (last > prev) {
              acc_j[1] = j;
              acc_ps[1] = last;
              add_pair(fin, a0, j);
              prev = last;
              new_pos = pos + j + 1;
              if (ws.refresh_every > 0 && (n_acc + 1) % ws.refresh_every == 0) nw.halt = 1;
              if (ws.stop_enabled && prev - ws.init_psnr >= ws.stop_diff) stop = true;
              n_acc += 1;
              break;
            }
          }
        }
      }
      HBX_TT(10);
      // apply the accepts: mask bits, group sums, log, commits for the next launch
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int j = acc_j[s2];
        if (j < 0) break;
        const WalkCand cj = s_cd[j];
        const size_t mw = ((size_t)cj.ch * N + cj.r) * (N / 64) + cj.col / 64;
        // device-scope atomic, performed past the XCD L2s (the persistent walk's readers load
        // mask words with sc1; tests/test_gpu_parity.py::test_walk_repeated_positions_* revisits them)
        atomicXor(reinterpret_cast<unsigned long long*>(a.mask) + mw, 1ull << (cj.col & 63));   // DBS_1024_24.py:320
        const int64_t n = ws.accepted + s2;
        if (n < a.log_cap) {
          a.log_pos[n] = pos + j;
          a.log_psnr[n] = acc_ps[s2];
        }
        if (s2 == 0) { nw.commit_ch = cj.ch; nw.commit_pix = cj.pix; }
        else { nw.commit2_ch1 = cj.ch + 1; nw.commit_pix2 = cj.pix; }
      }
#pragma unroll
      for (int i = 0; i < 3 * NG; ++i)
        if (i < 3 * G) {                                                           // :358-363
          if constexpr (PERSIST)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(walk_u32x2, fin[i]), r_bs, i * 8, 0, kSc1);
          else
            a.base_stats[i] = fin[i];
        }
    }
    nw.accepted = n_acc;
    nw.prev_psnr = prev;
    if (!isnan(last)) nw.last_psnr = last;
    nw.pos = new_pos;
    if (stop) { nw.done = 1; nw.stopped_early = 1; }
    if (nw.pos >= total) nw.done = 1;
  }
  HBX_TT(11);
  // the next launch's actions and signs (the bits this batch flipped toggled)
  WalkPre np;
  np.pos = kv > 0 ? new_pos : -1;        // a commit-only launch decodes nothing
  np.order = a.order;
  np.n = 0;
  np.pad = 0;
  const int base = (int)(new_pos - pos - 1);
#pragma unroll
  for (int j = 0; j < kWalkPreMax; ++j) {
    const int i = base + j;
    const bool have = i >= 0 && i < nn;
    const int ch = have ? s_nch[i] : -1, pix = have ? s_npix[i] : 0;
    const uint64_t wd = have ? s_nwd[i] : 0;
    np.ch[j] = ch;
    np.pix[j] = pix;
    if (have) np.n = j + 1;
    const bool ok = ch >= 0;
    int bit = (int)((wd >> ((pix % N) & 63)) & 1ull);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
      if (acc_j[s2] >= 0) {
        const WalkCand cj = s_cd[acc_j[s2]];
        if (cj.ch == ch && cj.pix == pix) bit ^= 1;
      }
    np.delta[j] = ok ? a.vb * (float)(1 - 2 * bit) : 0.0f;
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    np.cdelta[s2] = acc_j[s2] >= 0 ? s_cd[acc_j[s2]].delta : 0.0f;   // vb (2 bit' - 1) = vb (1 - 2 bit)
  if constexpr (PERSIST) {   // staged: the block's lanes store them write-through below, one word each
    s_ws = nw;
    s_pre = np;
  } else {
    *prep = np;
    *w = nw;
  }
#ifdef HBX_WALK_TIMING
  HBX_TT(7);
  if (nw.batches % 500 == 7) {
    const unsigned long long t00 = tt[0];
    printf("walk_step K %d batch %ld pre %d (10ns ticks from the deciding block's start): decider start %lld, state %lld, decode %lld, "
           "pixels %lld, blocksum %lld, arrival %lld, gather %lld, sum2 %lld, psnr %lld, decided %lld, applied %lld, end %lld\n", K, (long)nw.batches,
           (int)use_pre, (long long)(tt[0] - t00), (long long)(tt[8] - t00), (long long)(tt[1] - t00), (long long)(tt[2] - t00),
           (long long)(tt[3] - t00), (long long)(tt[4] - t00), (long long)(tt[5] - t00), (long long)(tt[6] - t00),
           (long long)(tt[9] - t00), (long long)(tt[10] - t00), (long long)(tt[11] - t00), (long long)(tt[7] - t00));
    if (NT * gridDim.x + 2 * gridDim.x <= 6656) {
      const long long* dbg = reinterpret_cast<const long long*>(a.partial + NT * gridDim.x);
      long long s0 = 1ll << 62, s1 = -(1ll << 62), l0 = 1ll << 62, l1 = 0, lsum = 0;
      int nslow = 0;
      for (int b = 0; b < (int)gridDim.x; ++b) {
        const long long st = __hip_atomic_load(dbg + 2 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (long long)t00;
        const long long la = __hip_atomic_load(dbg + 2 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s0 = st < s0 ? st : s0; s1 = st > s1 ? st : s1;
        l0 = la < l0 ? la : l0; l1 = la > l1 ? la : l1; lsum += la;
        nslow += la > 1000;
      }
      printf("   blocks: start [%lld, %lld], state latency min %lld max %lld mean %lld, >10us: %d\n", s0, s1, l0, l1,
             lsum / (long long)gridDim.x, nslow);
    }
  }
#endif
  }   // tid == 0
  if constexpr (!PERSIST) {
    return;
  } else {
    // a waiting block that times out raises the abort word (and stores fault = done = 1, which
    // this block's state store below may overwrite): k_walk_abort_fold, queued behind the
    // launch, folds the abort word into the state after every block has finished
    __syncthreads();
    if (tid < kWsWords)
      __builtin_amdgcn_raw_buffer_store_b32(reinterpret_cast<const unsigned*>(&s_ws)[tid], r_ws, tid * 4, 0, kSc1);
    else if (tid < kWsWords + kPreWords)
      __builtin_amdgcn_raw_buffer_store_b32(reinterpret_cast<const unsigned*>(&s_pre)[tid - kWsWords], r_pre,
                                            (tid - kWsWords) * 4, 0, kSc1);
    // every write-through store and atomic of the decision (mask word, statistics, state, next
    // actions, ticket reset) retired before the generation bump releases the other blocks
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(gen, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_gen = s_gen + 1;
    }
    __syncthreads();
  }
  }   // batch loop
}

// after a persistent launch: a timed-out grid barrier (abort word) marks the walk state faulted
// and done, whatever the deciding block stored last (runs once the grid has drained)
__global__ void k_walk_abort_fold(const int* abort_word, hbx_dbs_walk_t* w) {
  if (threadIdx.x == 0 && *abort_word) {
    w->fault = 1;
    w->done = 1;
  }
}

// blocks per candidate: enough blocks in flight to stream at full rate for
// small K, never more than one quad per thread
int walk_blocks_per_job(int N, int K) {
  const int nq = N * N / 4;
  const int max_b = (nq + kWalkNT - 1) / kWalkNT;
  int b = 1;
  while (b * K < 2048 && b < 1024) b *= 2;
  return b < max_b ? b : max_b;
}

// fused-step variants: K = 1 (single accept), 2..4 (two accepts resolved per batch);
// other K run the split three-kernel batch (a fused step keeps every candidate's
// loads of a quad in registers: beyond 4 candidates that spills)
bool walk_fused_k(int K) { return K >= 1 && K <= 4; }

int walk_step_blocks(int N) {
  const int nq = N * N / 4;
  const int b = (nq + kWalkNT - 1) / kWalkNT;          // one quad per thread at most
  return b < kWalkStepBlocksMax ? b : kWalkStepBlocksMax;
}

hipError_t launch_walk(const PlanDev& pd, const WalkLaunch& l, hipStream_t st) {
  WalkArgs a;
  a.mask = l.mask;
  a.target = l.target;
  a.base_stats = l.base_stats;
  a.field = l.field;
  a.inten = l.inten;
  a.order = l.order;
  a.n_order = l.n_order;
  a.w = l.walk;
  a.log_pos = l.log_pos;
  a.log_psnr = l.log_psnr;
  a.log_cap = l.log_cap;
  a.hpsf = pd.hpsf;
  a.partial = l.partial;
  a.N = pd.N;
  a.P = pd.P;
  a.G = pd.G;
  a.K = l.K;
  a.bpj = walk_blocks_per_job(pd.N, l.K);
  a.vb = pd.vb;
  a.count = l.count;
  a.peak = l.peak;
  a.rel = l.rel;
  a.commit_only = 0;
  const int nq = pd.N * pd.N / 4;
  const dim3 grid((unsigned)walk_step_blocks(pd.N));
  if (l.fused && walk_fused_k(l.K)) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st, &cap);   // graph capture: per-batch launches (no cooperative node)
    if (l.persist && l.batches > 1 && cap == hipStreamCaptureStatusNone) {
      // one cooperative launch for the whole call (co-residency of the grid guaranteed, or the
      // launch fails and the call falls back to one launch per batch below)
      int nb = l.batches;
      void* args[] = {&a, (void*)&l.counter, &nb};
      const void* fn = nullptr;
      switch (l.K) {
        case 1: fn = reinterpret_cast<const void*>(&k_walk_step<1, false, true>); break;
        case 2: fn = reinterpret_cast<const void*>(&k_walk_step<2, true, true>); break;
        case 3: fn = reinterpret_cast<const void*>(&k_walk_step<3, true, true>); break;
        default: fn = reinterpret_cast<const void*>(&k_walk_step<4, true, true>); break;
      }
      if (hipLaunchCooperativeKernel(fn, grid, dim3(kWalkNT), args, 0, st) == hipSuccess) {
        // the abort word goes into the walk state only once the whole grid has drained (stream
        // order): a decider that stored its state after a waiter's timeout cannot hide it
        hipLaunchKernelGGL(k_walk_abort_fold, dim3(1), dim3(64), 0, st, l.counter + kWalkAbort, l.walk);
        return hipGetLastError();
      }
      (void)hipGetLastError();
    }
    for (int b = 0; b < l.batches; ++b) {
      switch (l.K) {
        case 1: hipLaunchKernelGGL((k_walk_step<1, false, false>), grid, dim3(kWalkNT), 0, st, a, l.counter, 1); break;
        case 2: hipLaunchKernelGGL((k_walk_step<2, true, false>), grid, dim3(kWalkNT), 0, st, a, l.counter, 1); break;
        case 3: hipLaunchKernelGGL((k_walk_step<3, true, false>), grid, dim3(kWalkNT), 0, st, a, l.counter, 1); break;
        default: hipLaunchKernelGGL((k_walk_step<4, true, false>), grid, dim3(kWalkNT), 0, st, a, l.counter, 1); break;
      }
    }
    return hipGetLastError();
  }
  const unsigned bpc = (unsigned)std::min(512, (nq + kWalkNT - 1) / kWalkNT);
  if (l.fused && l.batches > 0) {
    // commits a fused step left pending (the split eval reads field / intensity as they
    // are): one commit-only step, which returns at once when there are none
    WalkArgs c = a;
    c.commit_only = 1;
    hipLaunchKernelGGL((k_walk_step<1, false, false>), grid, dim3(kWalkNT), 0, st, c, l.counter, 1);
  }
  for (int b = 0; b < l.batches; ++b) {
    hipLaunchKernelGGL(k_walk_eval, dim3((unsigned)a.bpj, (unsigned)l.K), dim3(kWalkNT), 0, st, a);
    hipLaunchKernelGGL(k_walk_decide, dim3(1), dim3(kWalkNT), 0, st, a);
    hipLaunchKernelGGL(k_walk_commit, dim3(bpc), dim3(kWalkNT), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace hbx
