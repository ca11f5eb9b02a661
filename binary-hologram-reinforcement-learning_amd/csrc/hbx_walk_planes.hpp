// hbx_walk_planes.hpp -- the decision of the FFT-mode greedy walk on the plane cache
// (hbx_dbs_walk_planes, ABI v10), shared by the stand-alone k_walk_planes (hbx_kernels.hip) and,
// since r05, the last-arriving workgroup of the walk's k_rowinv_d launch (hbx_passes.hip), which
// decides right after the batch's partials are in instead of in a launch of its own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hbx.h"
#include "hbx_internal.hpp"

namespace hbx {

constexpr int kWalkPlanesCJ = 8;             // jobs per staging round of the partials
constexpr int kSc1Bit = 16;                  // buffer cache policy sc1 (gfx950): write-through / L2-fresh
constexpr int kFillRejected = -2;            // job of a candidate the on-pixel constraint rejects (the
                                             // passes skip every env < 0; the decision keeps its group)

// LDS the decision needs for RB row blocks per job (carved out of a caller's buffer)
__host__ __device__ constexpr size_t walk_planes_lds_bytes(int RB) {
  return (size_t)kWalkPlanesCJ * 3 * RB * 8 + 256 * 3 * 8 + 256 * sizeof(JobDesc) + 256 * 8 + 256 * 4 * 4 +
         512 * 8 + 3 * HBX_MAX_GROUPS * 8 + 128 + HBX_MAX_GROUPS * 8 + 16;
}

// (ABI v13, extension -- no reference counterpart) the on-pixel ratio constraint: a
// flip moving group g's on-pixel count C by d = +-1 is admissible iff |C + d - T| <= tol or it
// brings C closer to the target T.  hbx/dbs.py fill_admissible and oracle/hbx_oracle.py carry the
// same rule.
__host__ __device__ __forceinline__ bool fill_admissible(int64_t count, int64_t target, int64_t tol, int bit) {
  const int64_t d = bit ? -1 : 1;
  const int64_t now = count - target < 0 ? target - count : count - target;
  const int64_t after = count + d - target < 0 ? target - count - d : count + d - target;
  return after <= tol || after < now;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t walk_planes_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, (int)bytes,
                                           0x00020000);
}

// The decision, by one 256-thread block.  decide = 1: the candidates of the batch just propagated
// (jobs[c] = order[pos + c], each propagated against the batch's base state) are visited in order
// by one thread, exactly as the serial loop (DBS_1024_24.py:313-363) visits them: a candidate's
// PSNR is formed from its group's propagated stats and the CURRENT stats of the other groups
// (k_eval_finalize's sum order), and the first strict improvement (:355) is committed as
// hbx_commit_flip_planes does (mask bit, group stats, prev PSNR, the pair's spare slots swapped
// in) and logged.  The visit then CONTINUES: a later candidate of a colour group no accept of
// this batch has touched was propagated against exactly the group state the serial loop would
// propagate it against (the other groups enter only through their stats), so its PSNR is the
// serial loop's bit for bit; the batch ends before the first candidate of a touched group (it
// needs a fresh propagation) -- up to G accepts per batch.  Then -- decide = 0 too -- the NEXT
// batch's K jobs are written from the walk state (invalid jobs once the walk is done, so the
// passes behind return at once).  (r06) With a ring / phase buffer (the fused walk), candidate i of
// a batch sits in job slot (ring + i) % K: the candidates this batch propagated but did not visit
// stay in their slots as the next batch's first candidates, and phase[slot] tells the passes what
// they still need (0 all, 1 only k_rowinv_d, 2 nothing; see WalkPlanesArgs).  SC1: the partials come from other workgroups of the SAME launch
// (the fused decision), written through with sc1 stores -- read them with sc1 loads, which miss
// this XCD's L2.
template <bool SC1>
__device__ __forceinline__ void walk_planes_decide(const WalkPlanesArgs& a, int decide, char* lds) {
  const int RB = a.RB, K = a.K, G = a.G, P = a.P, H = a.H, W = a.W;
  constexpr int CJ = kWalkPlanesCJ;
  char* q = lds;
  auto carve = [&](size_t bytes) { char* r = q; q += (bytes + 7) & ~(size_t)7; return r; };
  double* s_part = reinterpret_cast<double*>(carve((size_t)CJ * 3 * RB * 8));
  double* s_js = reinterpret_cast<double*>(carve(256 * 3 * 8));
  JobDesc* s_job = reinterpret_cast<JobDesc*>(carve(256 * sizeof(JobDesc)));
  uint64_t* s_word = reinterpret_cast<uint64_t*>(carve(256 * 8));
  int32_t* s_slot = reinterpret_cast<int32_t*>(carve(256 * 4 * 4));   // [c][4]
  int64_t* s_order = reinterpret_cast<int64_t*>(carve(512 * 8));
  double* s_base = reinterpret_cast<double*>(carve(3 * HBX_MAX_GROUPS * 8));
  int64_t* s_i64 = reinterpret_cast<int64_t*>(carve(3 * 8));           // pos, total, acc
  int* s_int = reinterpret_cast<int*>(carve(4 * 4));                    // done, stop_en, ring, -
  double* s_dbl = reinterpret_cast<double*>(carve(4 * 8));              // prev, last, init, stop_diff
  int64_t* s_fill = reinterpret_cast<int64_t*>(carve(HBX_MAX_GROUPS * 8));   // on-pixel counts (fill on)
  uint64_t* s_tpair = reinterpret_cast<uint64_t*>(carve(8));            // (group, pair)s this batch accepted into
  hbx_dbs_walk_t* w = a.w;
  const int k = threadIdx.x;
  const int64_t hw = (int64_t)H * W;
  const int CH = G * P;
  // (r05) every load that depends on nothing goes out first, together: the walk position (read by
  // every lane: one broadcast load, so the order window needs no block barrier), the candidates'
  // jobs, the base statistics and the first partials; then the loads that depend on them (the
  // order window, each candidate's mask word and slot pairs).  The r04 form chained them through
  // block barriers -- 11 us per decision, now the latency of two dependent loads plus the sums.
  const int64_t pos0 = w->pos, total0 = w->total;
  JobDesc jb_k;
  jb_k.env = -1;
  if (decide && k < K) jb_k = a.jobs[k];
  if (decide && k < 3 * G) s_base[k] = a.base_stats[k];
  if (a.fill_count && k < G) s_fill[k] = a.fill_count[k];
  const __amdgpu_buffer_rsrc_t rp = walk_planes_rsrc(a.partial, (unsigned)((size_t)K * RB * 3 * 8));
  constexpr int PRE = 8;                    // partials per lane issued up front (first chunk)
  double pre[PRE];
  const int n0 = (K < CJ ? K : CJ) * RB * 3;
  if (decide) {
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int i = k + u * (int)blockDim.x;
      if (i < n0) {
        if constexpr (SC1)
          pre[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rp, i * 8, 0, kSc1Bit));
        else
          pre[u] = a.partial[i];
      }
    }
  }
  // (r06) retention: candidate i of the batch sits in job slot (ring + i) % K; a call's first batch
  // (decide = 0) starts at ring 0 with every slot propagated in full
  const bool keep = a.phase != nullptr && a.ring != nullptr;
  if (k == 0) {
    s_i64[0] = pos0; s_i64[1] = total0; s_i64[2] = w->accepted; s_int[0] = w->done;
    s_int[1] = w->stop_enabled; s_dbl[0] = w->prev_psnr; s_dbl[1] = w->last_psnr;
    s_dbl[2] = w->init_psnr; s_dbl[3] = w->stop_diff;
    s_int[2] = (keep && decide) ? *a.ring : 0;
    s_tpair[0] = 0;
  }
  for (int i = k; i < 2 * K; i += blockDim.x) s_order[i] = (pos0 + i < total0) ? a.order[pos0 + i] : -1;
  if (decide && k < K) {
    s_job[k] = jb_k;
    if (jb_k.env >= 0) {
      const int ch = jb_k.group * P + jb_k.flip_plane;
      s_word[k] = a.mask[(size_t)ch * H * (W / 64) + (size_t)(jb_k.flip_pix / W) * (W / 64) + (jb_k.flip_pix % W) / 64];
      const int pa = jb_k.group * P + (jb_k.flip_plane & ~1);
      s_slot[4 * k + 0] = a.plane_slot[pa];
      s_slot[4 * k + 1] = a.plane_slot[pa + 1];
      s_slot[4 * k + 2] = a.plane_slot[CH + 2 * k];
      s_slot[4 * k + 3] = a.plane_slot[CH + 2 * k + 1];
    }
  }
  if (decide) {
    // each candidate's three statistics summed over its row blocks in row-block order,
    // k_reduce_partials' order bit for bit
    for (int c0 = 0; c0 < K; c0 += CJ) {
      const int nj = K - c0 < CJ ? K - c0 : CJ;
      if (c0 == 0) {
        const bool fits = n0 <= PRE * (int)blockDim.x;
#pragma unroll
        for (int u = 0; u < PRE; ++u) {
          const int i = k + u * (int)blockDim.x;
          if (i < n0) s_part[i] = pre[u];
        }
        if (!fits)
          for (int i = k + PRE * (int)blockDim.x; i < n0; i += blockDim.x)
            s_part[i] = SC1 ? __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rp, i * 8, 0, kSc1Bit))
                            : a.partial[i];
      } else {
        for (int i = k; i < nj * RB * 3; i += blockDim.x) {
          if constexpr (SC1)
            s_part[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                       rp, (int)(((size_t)c0 * RB * 3 + i) * 8), 0, kSc1Bit));
          else
            s_part[i] = a.partial[(size_t)c0 * RB * 3 + i];
        }
      }
      __syncthreads();
      if (k < nj * 3) {
        const int c = k / 3, st = k % 3;
        double acc = 0.0;
        // unrolled: the LDS loads of 16 terms go out back to back ahead of the (in-order) adds;
        // the rolled loop waited one LDS round trip per term (~128 x 120 cycles per statistic)
#pragma unroll 16
        for (int i = st; i < 3 * RB; i += 3) acc += s_part[c * 3 * RB + i];
        s_js[3 * (c0 + c) + st] = acc;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (k == 0 && decide && !s_int[0]) {
    const int64_t pos = s_i64[0];
    const int nk = (int)min((int64_t)K, s_i64[1] - pos);
    const int ring = s_int[2];
    double prev = s_dbl[0], last = s_dbl[1];
    int64_t acc_n = s_i64[2];
    unsigned touched = 0;
    uint64_t tpair = 0;
    int visited = nk, done = 0;
    for (int i = 0; i < nk; ++i) {
      const int c = (ring + i) % K;         // candidate i's job slot
      const JobDesc jb = s_job[c];
      // (an inadmissible candidate, env == kFillRejected, was judged against the batch's starting
      // count: it ends the batch like any other candidate of a touched group)
      if (jb.env != -1 && ((touched >> jb.group) & 1u)) { visited = i; break; }
      double ps = NAN;
      const double* js = s_js + 3 * c;
      if (jb.env >= 0) {
        double sxy = 0.0, sxx = 0.0, syy = 0.0;
        for (int gg = 0; gg < G; ++gg) {    // k_eval_finalize's sum order
          if (gg == jb.group) { sxy += js[0]; sxx += js[1]; syy += js[2]; }
          else { sxy += s_base[3 * gg]; sxx += s_base[3 * gg + 1]; syy += s_base[3 * gg + 2]; }
        }
        ps = psnr_from(sxy, sxx, syy, a.count, a.rel_scale, a.peak);
      }
      last = ps;
      if (ps > prev) {                     // commit candidate c
        const int ch = jb.group * P + jb.flip_plane;
        const int pix = jb.flip_pix;
        a.mask[(size_t)ch * H * (W / 64) + (size_t)(pix / W) * (W / 64) + (pix % W) / 64] =
            s_word[c] ^ (1ull << ((pix % W) & 63));
        s_base[3 * jb.group] = js[0];
        s_base[3 * jb.group + 1] = js[1];
        s_base[3 * jb.group + 2] = js[2];
        a.base_stats[3 * jb.group] = js[0];
        a.base_stats[3 * jb.group + 1] = js[1];
        a.base_stats[3 * jb.group + 2] = js[2];
        const int pa = jb.group * P + (jb.flip_plane & ~1);
        a.plane_slot[pa] = s_slot[4 * c + 2];        // the fresh pair's slots become current,
        a.plane_slot[pa + 1] = s_slot[4 * c + 3];
        a.plane_slot[CH + 2 * c] = s_slot[4 * c + 0];    // the replaced ones become spares
        a.plane_slot[CH + 2 * c + 1] = s_slot[4 * c + 1];
        if (a.fill_count) {                  // the accepted flip's move of its group's on-pixel count
          const int64_t f = s_fill[jb.group] + (((s_word[c] >> ((pix % W) & 63)) & 1ull) ? -1 : 1);
          s_fill[jb.group] = f;
          a.fill_count[jb.group] = f;
        }
        if (acc_n < a.accept_cap) { a.accept_pos[acc_n] = pos + i; a.accept_psnr[acc_n] = ps; }
        ++acc_n;
        prev = ps;
        touched |= 1u << jb.group;
        tpair |= 1ull << ((jb.group * P + jb.flip_plane) >> 1);
        if (s_int[1] && ps - s_dbl[2] >= s_dbl[3]) {   // DBS_ratio_0.5.py:366-372
          done = 1;
          w->stopped_early = 1;
          visited = i + 1;
          break;
        }
      }
    }
    s_tpair[0] = tpair | ((uint64_t)touched << 48);   // pairs (bits < 48) and groups
    w->accepted = acc_n;
    w->prev_psnr = prev;
    w->last_psnr = last;
    w->pos = pos + visited;
    w->batches += 1;
    const int d = (done || pos + visited >= s_i64[1]) ? 1 : 0;
    if (d) w->done = 1;
    s_int[0] = d;
    s_i64[2] = visited;                      // reused: the next batch's offset in the order window
  } else if (k == 0) {
    s_i64[2] = 0;
  }
  __syncthreads();
  if (k < K) {                              // the next batch's jobs
    const int off = (int)s_i64[2];
    const int64_t qq = s_i64[0] + off + k;
    // candidate k of the next batch: job slot (ring + off + k) % K with retention (the slot the
    // same candidate had in this batch when k < K - off), slot k without
    const int slot = keep ? (s_int[2] + off + k) % K : k;
    JobDesc jd;
    jd.env = -1; jd.group = 0; jd.flip_plane = -1; jd.flip_pix = 0;
    if (!s_int[0] && qq < s_i64[1]) {
      const int64_t av = s_order[off + k];
      if (av >= 0 && av < (int64_t)G * P * hw) {
        const int ch = (int)(av / hw);
        jd.env = 0; jd.group = ch / P; jd.flip_plane = ch % P; jd.flip_pix = (int)(av % hw);
        if (a.fill_count) {
          // an inadmissible candidate is visited and rejected without a propagation: a job the
          // passes skip (no PSNR).  The counts are this decision's; an earlier accept of the next
          // batch in the same group ends that batch at this candidate, which is then re-issued
          // against the updated count
          const int pix = jd.flip_pix;
          const uint64_t word = a.mask[(size_t)ch * H * (W / 64) + (size_t)(pix / W) * (W / 64) + (pix % W) / 64];
          if (!fill_admissible(s_fill[jd.group], a.fill_target, a.fill_tol, (int)((word >> ((pix % W) & 63)) & 1ull)))
            jd.env = kFillRejected;
        }
      }
    }
    if (keep) {
      // what the slot still needs: a candidate this batch propagated (same slot, k < K - off) keeps
      // its pair's B unless an accept of this batch changed that pair's mask, and keeps its
      // partials and fresh pair too unless an accept changed its colour group's cached planes
      uint8_t ph = 0;
      const JobDesc old = s_job[slot];
      if (decide && off > 0 && k < K - off && jd.env >= 0 && old.env >= 0) {
        const uint64_t tp = s_tpair[0];
        if (!((tp >> ((jd.group * P + jd.flip_plane) >> 1)) & 1ull))
          ph = ((tp >> (48 + jd.group)) & 1ull) ? 1 : 2;
      }
      a.phase[slot] = ph;
    }
    a.jobs[slot] = jd;
  }
  if (keep && k == 0) *a.ring = decide ? (s_int[2] + (int)s_i64[2]) % K : 0;
}

// The fused decision's hand-off, at the end of every k_rowinv_d workgroup of a walk batch: this
// block's partials went out write-through (sc1) and have retired (s_waitcnt vmcnt(0)); one
// agent-scope ticket per block; the block holding the last ticket resets the counter for the next
// launch and decides (the psf walk's recipe, hbx_walk.hip k_walk_step: relaxed ticket + sc1 loads,
// pinned to gfx950's cache policy, every walk test checks the accept sequence against the oracle).
__device__ __forceinline__ void walk_planes_arrive(const WalkPlanesArgs& a, char* lds) {
  __shared__ int s_last_block;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int got = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last_block = got == (int)(gridDim.x * gridDim.y * gridDim.z) - 1;
    if (s_last_block) __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_last_block) walk_planes_decide<true>(a, 1, lds);
}

}  // namespace hbx
