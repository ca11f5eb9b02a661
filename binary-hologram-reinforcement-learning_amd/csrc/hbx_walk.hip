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
    if (threadIdx.x == 0) w->commit_ch = -1;
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
    nw.commit_ch = ch;
    nw.commit_pix = pix;
    nw.pos = pos + acc + 1;
    if (ws.stop_enabled && ps - ws.init_psnr >= ws.stop_diff) {   // DBS_ratio_0.5.py:366-372
      nw.done = 1;
      nw.stopped_early = 1;
    }
    if (ws.refresh_every > 0 && (n + 1) % ws.refresh_every == 0) nw.halt = 1;
  } else {
    if (kv > 0) nw.last_psnr = s_ps[kv - 1];
    nw.commit_ch = -1;
    nw.pos = pos + kv;
  }
  if (nw.pos >= total) nw.done = 1;
  *w = nw;
}

// the accepted flip of the batch (mask bit already toggled): U_c += delta h,
// I_g += (|U_c'|^2 - |U_c|^2) / P
__global__ __launch_bounds__(kWalkNT) void k_walk_commit(WalkArgs a) {
  hbx_dbs_walk_t* w = a.w;
  const int ch = w->commit_ch;
  if (ch < 0) return;
  const int pix = w->commit_pix;
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

// blocks per candidate: enough blocks in flight to stream at full rate for
// small K, never more than one quad per thread
int walk_blocks_per_job(int N, int K) {
  const int nq = N * N / 4;
  const int max_b = (nq + kWalkNT - 1) / kWalkNT;
  int b = 1;
  while (b * K < 2048 && b < 1024) b *= 2;
  return b < max_b ? b : max_b;
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
  const int nq = pd.N * pd.N / 4;
  const unsigned bpc = (unsigned)std::min(512, (nq + kWalkNT - 1) / kWalkNT);
  for (int b = 0; b < l.batches; ++b) {
    hipLaunchKernelGGL(k_walk_eval, dim3((unsigned)a.bpj, (unsigned)l.K), dim3(kWalkNT), 0, st, a);
    hipLaunchKernelGGL(k_walk_decide, dim3(1), dim3(kWalkNT), 0, st, a);
    hipLaunchKernelGGL(k_walk_commit, dim3(bpc), dim3(kWalkNT), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace hbx
