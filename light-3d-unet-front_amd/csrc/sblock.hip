// Whole ResidualBlock forward at small volumes in ONE launch (the 6^3 level of the shipped
// network: down3 64->128 with its Conv1x1 shortcut, bottleneck 128->128).  Replaces
// ResidualBlock.forward (light_unet/models/unet3d.py:77-93) with DepthwiseSeparableConv3d convs
// (unet3d.py:10-23) -- five launches of a few microseconds each in the level-by-level schedule
// (depthwise, pointwise(+shortcut), depthwise, pointwise, tail), each one latency-bound at
// 4 x 128 x 216 voxels.
//
// Mapping (gfx950): workgroup (n, g), 1024 threads, owns output channels 16g..16g+15 of sample n
// (G = Cout/16 workgroups per sample; N*G <= 256, all resident).  Everything a channel's
// InstanceNorm needs (all S <= 256 voxels) lives in the workgroup, so statistics, records and
// the normalise/activate/dropout are local; only the two pointwise contractions read every
// channel of the sample, so the sample's G workgroups meet at two barriers:
//   1  depthwise conv1 of this workgroup's Cin/G input channels -> z1 (global)
//   -- sample barrier --
//   2  z1 (all Cin) [+ x for the shortcut] -> LDS; MFMA contraction of the 16-channel rows
//      y1 = W1 z1 [, r = Wsc x]  -> y1 / r (global) and LDS tiles
//   3  InstanceNorm statistics (fp64, exact per channel), records rec1 (with Dropout3d) / rec_r
//   4  a1 = lrelu(IN1(y1)) * keep into zero-haloed LDS images; depthwise conv2 -> z2 (global)
//   -- sample barrier --
//   5  z2 (all Cout) -> LDS; y2 = W2 z2 -> y2 (global); statistics -> rec2
//   6  out = lrelu(IN2(y2) + (IN_sc(r) or x))
// The contractions use v_mfma_f32_16x16x4f32 on [16 channels] x [16-voxel tiles]; LDS rows are
// padded to SP = 16*ntile + 8 floats so the four k-rows of an MFMA B read hit disjoint banks.
// Barrier: a monotonic per-sample arrival counter (no reset between launches or graph replays;
// agent-scope release/acquire so the other XCDs' L2s see z1 / z2); the spin is bounded and a
// timeout is flagged in sync[N] instead of hanging the device.
#include "common.h"
using namespace l3u;

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 1024, kWaves = 16;

L3U_DEV f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

L3U_DEV float rnd(float v, const float*) { return v; }
L3U_DEV float rnd(float v, const bf16*) { return (float)(bf16)v; }

// All G workgroups of one sample arrive, then all leave.  ctr counts arrivals monotonically:
// the arrival that returns `old` belongs to the episode ending at the next multiple of G.
L3U_DEV void sample_barrier(unsigned* ctr, unsigned G, unsigned* err) {
  // every wave's global stores have reached L2 before thread 0's agent-scope release writes L2
  // back (a workgroup-scope __syncthreads does not wait for them)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (old / G + 1) * G;
    int spins = 0;
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) {   // ~ a second: flag it and let the grid drain
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every outstanding
// global store of the wave (a full memory round trip per stage here); the stores of z / y / r
// drain in the background instead, and the sample barrier's release fence orders them.
L3U_DEV void bar_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct SbGeom {
  int S, SP, ntile, P3, zrows, wreg;
  size_t lds;   // bytes
  bool ok;
};

L3U_INLINE_HOST SbGeom sb_geom(int Cin, int Cout, int D, int H, int W, int sc) {
  SbGeom g{};
  g.ok = false;
  if (Cin < 1 || Cout < 16 || Cout % 16 != 0 || Cout > 128 || Cin > 128 || Cin % 4 != 0) return g;
  if (D < 1 || H < 1 || W < 1) return g;
  const int G = Cout / 16;
  if (Cin % G != 0 || Cin / G > 16) return g;
  if (!sc && Cin != Cout) return g;
  g.S = D * H * W;
  if (g.S > 256 || g.S < 4) return g;
  g.ntile = (g.S + 15) / 16;
  g.SP = 16 * g.ntile + 8;
  g.P3 = (D + 2) * (H + 2) * (W + 2);
  const int zrows = max(Cin * (1 + sc), Cout);
  g.zrows = max(zrows, (16 * g.P3 + g.SP - 1) / g.SP);   // the halo images alias this region
  g.wreg = max((1 + sc) * 16 * (Cin + 4), 16 * (Cout + 4));
  const int un = max(16 * 27, 2 * g.ntile * 16 * 2);
  // Z region + y / r tiles + 3 x 16 records + A-operand rows + taps / tile statistics
  g.lds = ((size_t)g.zrows * g.SP + 2 * 16 * g.SP + 3 * 16 * kRec + g.wreg + un) * sizeof(float);
  if (g.lds > 160 * 1024) return g;
  g.ok = true;
  return g;
}

// workgroups launched (sample octets x G; see sb_map)
L3U_INLINE_HOST int sb_blocks(int N, int Cout) { return (N + 7) / 8 * 8 * (Cout / 16); }

// rows x S elements of src (row stride S) -> put(row, v, value): VW-wide loads, up to 4 per
// thread in flight before any is consumed (a load -> store chain per element costs one memory
// latency per iteration: measured 70 us per launch)
template <int VW, typename T, typename Put>
L3U_DEV void stage_rows(const T* src, int rows, int S, Put put) {
  constexpr int UB = 4;
  const int total = rows * S / VW;
  for (int i0 = threadIdx.x; i0 < total; i0 += kThreads * UB) {
    f4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = min(i0 + u * kThreads, total - 1);
      if constexpr (VW == 4) v[u] = ldv4(src + 4 * i);
      else v[u] = f4{ld1(src + i), 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = i0 + u * kThreads;
      if (i < total) {
        const int e = VW * i, c = e / S, vv = e - c * S;
#pragma unroll
        for (int q = 0; q < VW; ++q) put(c, vv + q, v[u][q]);
      }
    }
  }
}

// Workgroup b -> (sample, channel group): the G workgroups of a sample share b % 8, i.e. one XCD
// under the round-robin dispatch, so the z1 / z2 exchange reads hit that XCD's L2 (correctness
// does not depend on it: the barrier is agent-scope).  Samples n >= N of the last octet exit.
L3U_DEV void sb_map(int b, int G, int& n, int& g) {
  const int k = b >> 3;
  n = (k / G) * 8 + (b & 7);
  g = k % G;
}

// VW: 4 when S % 4 == 0 (float4 staging loads), else 1
template <typename T, int VW>
__global__ __launch_bounds__(kThreads) void sblock_fwd_kernel(l3u_sblock_fwd_args a, int N, int Cin,
                                                              int Cout, int D, int H, int W, int SP,
                                                              int ntile, int P3, int zrows, int wreg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int G = Cout / 16;
  int n, g;
  sb_map(blockIdx.x, G, n, g);
  if (n >= N) return;   // uniform: before any barrier
  const int row0 = 16 * g;
  const int S = D * H * W, HW = H * W, Wp = W + 2, HWp = (H + 2) * Wp, SV = 16 * ntile;
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63, lrm = l & 15, lk = l >> 4;
  const bool sc = a.w_sc != nullptr;
  float* zb = lds;                                   // [zrows][SP]: Z operands / halo images
  float* yt = zb + (size_t)zrows * SP;               // [16][SP]: y1, then y2
  float* rt = yt + 16 * SP;                          // [16][SP]: r
  float* rec = rt + 16 * SP;                         // [3][16][8]: rec_r, rec1, rec2
  float* wl = rec + 3 * 16 * kRec;                   // [roles][16][K + 4] MFMA A-operand rows
  float* un = wl + wreg;                             // taps1 | tile statistics | taps2 | ...
  float* taps = un;                                  //   [16][27]
  float* tst = un;                                   //   [2 roles][ntile][16 rows][mean, M2]
  const T* xn = reinterpret_cast<const T*>(a.x) + (long long)n * a.x_nstride;
  unsigned* ctr = a.sync + n;
  unsigned* err = a.sync + N;
#ifdef L3U_SB_PROF   // stage timestamps (tools/sbprof.py): sync[64 ..] as [blocks][16] u64
  unsigned long long* prof = reinterpret_cast<unsigned long long*>(a.sync + 64) + (n * G + g) * 16;
  int pk = 0;
#define SBP() do { if (tid == 0) prof[pk] = wall_clock64(); ++pk; } while (0)
#else
#define SBP() do {} while (0)
#endif
  SBP();

  // halo-image offset of voxel v (no divisions in the loops: a per-thread walk over i += 1024)
  auto img_off = [&](int v) {
    const int zz = v / HW, rem = v - zz * HW, yy = rem / W, xx = rem - yy * W;
    return ((zz + 1) * (H + 2) + yy + 1) * Wp + xx + 1;
  };
  const int jq = kThreads / S, jr = kThreads - jq * S;   // the walk's (channel, voxel) step
  // depthwise 3^3 of nch zero-haloed channel images in zb (taps in `taps`) -> dst channel rows
  auto dw_stage = [&](int nch, T* dst) {
    int c = tid / S, v = tid - c * S;
    for (int i = tid; i < nch * S; i += kThreads) {
      const float* im = zb + (size_t)c * P3 + img_off(v) - HWp - Wp - 1;
      const float* tw = taps + c * 27;
      float s = 0.f;
#pragma unroll
      for (int kz = 0; kz < 3; ++kz)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) s = fmaf(tw[kz * 9 + ky * 3 + kx], im[kz * HWp + ky * Wp + kx], s);
      st1(dst + i, s);
      c += jq;
      v += jr;
      if (v >= S) { v -= S; ++c; }
    }
  };
  auto zero_images = [&](int nch) {
    for (int i = tid; i < nch * P3; i += kThreads) zb[i] = 0.f;
  };
  auto zero_pad_cols = [&](int rows) {   // voxel columns S .. SV-1 of the contraction operand
    const int pc = SV - S;
    for (int i = tid; i < rows * pc; i += kThreads) zb[(i / pc) * SP + S + i % pc] = 0.f;
  };
  // rows row0 .. row0+15 of wm [.][K] -> wl role `role` (row stride K + 4: the 16 rows of one
  // MFMA A read spread over the banks)
  auto load_w = [&](const float* wm, int K, int role) {
    float* d = wl + role * 16 * (K + 4);
    for (int i = tid; i < 16 * K; i += kThreads) d[(i / K) * (K + 4) + i % K] = wm[(size_t)row0 * K + i];
  };
  // rows [k0, k0+K) of zb (the B operand) times A role `role` -> tile (16 x 16-voxel tile t),
  // dst rows, and the tile's per-row (mean, M2) over its valid voxels into tst[role][t]
  auto contract = [&](int t, int K, int k0, int role, float* tile, T* dst) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* br = zb + (size_t)(k0 + lk) * SP + 16 * t + lrm;
    const float* ar = wl + role * 16 * (K + 4) + lrm * (K + 4) + lk;
    for (int ks = 0; ks < K / 4; ks += 4) {
      float av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool in = ks + u < K / 4;
        av[u] = in ? ar[4 * (ks + u)] : 0.f;
        bv[u] = in ? br[(size_t)4 * (ks + u) * SP] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mfma4(av[u], bv[u], acc);
    }
    const int v = 16 * t + lrm;
    const bool ok = v < S;
    const float cnt = (float)min(16, S - 16 * t), inv = 1.f / cnt;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r = 4 * lk + rr;
      T* o = dst + (long long)r * S + v;
      const float q = rnd(acc[rr], o);
      tile[r * SP + v] = q;
      if (ok) st1(o, acc[rr]);
      // lanes of a DPP row share lk: the row's 16 voxels of this tile
      const float m = row_sum16(ok ? q : 0.f) * inv;
      const float d = ok ? q - m : 0.f;
      const float m2 = row_sum16(d * d);
      if (lrm == 0) {
        float* o2 = tst + ((role * ntile + t) * 16 + r) * 2;
        o2[0] = m;
        o2[1] = m2;
      }
    }
  };
  // records of rows 0..15 (role 0: y, role 1: r) from the tile statistics: thread r of the
  // role merges the tiles in order (Chan), as finalize_record merges GEMM partials
  auto records = [&](int role, const float* gm, const float* bt, float dp, int layer, float* lrec,
                     float* grec) {
    const int r = tid - role * 64;
    if (r >= 0 && r < 16) {
      float cn = 0.f, mu = 0.f, m2 = 0.f;
      for (int t = 0; t < ntile; ++t) {
        const float* p = tst + ((role * ntile + t) * 16 + r) * 2;
        chan_merge(cn, mu, m2, (float)min(16, S - 16 * t), p[0], p[1]);
      }
      l3u_norm_src s{};
      s.gamma = gm;
      s.beta = bt;
      s.drop_p = dp;
      s.layer = layer;
      s.seed = a.seed;
      s.step = a.step;
      float rc[kRec];
      record_from(s, n, row0 + r, Cout, cn, mu, m2, rc);
      float* go = grec + ((long long)n * Cout + row0 + r) * kRec;
#pragma unroll
      for (int i = 0; i < kRec; ++i) {
        lrec[r * kRec + i] = rc[i];
        go[i] = rc[i];
      }
    }
  };

  // ---- prefetch everything that does not depend on this launch's results: the identity
  // residual of the tail, conv2's taps and pointwise weights (registers), conv1's taps and
  // pointwise / shortcut weights (LDS)
  const int cpg = Cin / G, c0 = g * cpg;
  float xres[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) xres[q] = sc ? 0.f : ld1(xn + (long long)row0 * S + min(4 * tid + q, 16 * S - 1));
  const float tap2 = tid < 16 * 27 ? a.w_dw2[row0 * 27 + tid] : 0.f;
  float w2r[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * kThreads;
    w2r[u] = i < 16 * Cout ? a.w_pw2[(size_t)row0 * Cout + i] : 0.f;
  }
  zero_images(cpg);
  for (int i = tid; i < cpg * 27; i += kThreads) taps[i] = a.w_dw1[c0 * 27 + i];
  load_w(a.w_pw1, Cin, 0);
  if (sc) load_w(a.w_sc, Cin, 1);
  bar_lds();

  // ---- 1: depthwise conv1 of this workgroup's input channels
  stage_rows<VW>(xn + (long long)c0 * S, cpg, S,
                 [&](int c, int v, float val) { zb[(size_t)c * P3 + img_off(v)] = val; });
  bar_lds();
  SBP();
  T* z1n = reinterpret_cast<T*>(a.z1) + (long long)n * Cin * S;
  dw_stage(cpg, z1n + (long long)c0 * S);
  const bool rrole = sc && wv >= 8;
  SBP();
  sample_barrier(ctr, G, err);
  SBP();

  // ---- 2: pointwise conv1 (and the shortcut) over all input channels
  stage_rows<VW>(z1n, Cin, S, [&](int c, int v, float val) { zb[c * SP + v] = val; });
  if (sc) stage_rows<VW>(xn, Cin, S, [&](int c, int v, float val) { zb[(Cin + c) * SP + v] = val; });
  zero_pad_cols(Cin * (sc ? 2 : 1));
  bar_lds();
  SBP();
  T* y1n = reinterpret_cast<T*>(a.y1) + ((long long)n * Cout + row0) * S;
  T* rn = sc ? reinterpret_cast<T*>(a.r) + ((long long)n * Cout + row0) * S : nullptr;
  {
    const int wpr = sc ? 8 : 16, w0 = rrole ? wv - 8 : wv;
    for (int t = w0; t < ntile; t += wpr) {
      if (rrole) contract(t, Cin, Cin, 1, rt, rn);
      else contract(t, Cin, 0, 0, yt, y1n);
    }
  }
  bar_lds();
  SBP();
  // ---- 3: records of norm1 (Dropout3d) and the shortcut norm
  records(0, a.g1, a.b1, a.drop_p, a.layer1, rec + 16 * kRec, a.rec1);
  if (sc) records(1, a.g_sc, a.b_sc, 0.f, 0, rec, a.rec_r);
  bar_lds();
  SBP();

  // ---- 4: a1 = lrelu(IN1(y1)) * keep, depthwise conv2 of this workgroup's 16 channels
  zero_images(16);
  if (tid < 16 * 27) taps[tid] = tap2;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * kThreads;
    if (i < 16 * Cout) wl[(i / Cout) * (Cout + 4) + i % Cout] = w2r[u];
  }
  bar_lds();
  {
    int c = tid / S, v = tid - c * S;
    for (int i = tid; i < 16 * S; i += kThreads) {
      const float* rc = rec + (16 + c) * kRec;
      zb[(size_t)c * P3 + img_off(v)] = lrelu(fmaf(rc[2], yt[c * SP + v] - rc[0], rc[3]));
      c += jq;
      v += jr;
      if (v >= S) { v -= S; ++c; }
    }
  }
  bar_lds();
  T* z2n = reinterpret_cast<T*>(a.z2) + (long long)n * Cout * S;
  dw_stage(16, z2n + (long long)row0 * S);
  SBP();
  sample_barrier(ctr, G, err);   // also: every wave is done with the taps (tst aliases them)
  SBP();

  // ---- 5: pointwise conv2 over all channels, norm2 record
  stage_rows<VW>(z2n, Cout, S, [&](int c, int v, float val) { zb[c * SP + v] = val; });
  zero_pad_cols(Cout);
  bar_lds();
  SBP();
  T* y2n = reinterpret_cast<T*>(a.y2) + ((long long)n * Cout + row0) * S;
  for (int t = wv; t < ntile; t += kWaves) contract(t, Cout, 0, 0, yt, y2n);
  bar_lds();
  SBP();
  records(0, a.g2, a.b2, 0.f, 0, rec + 32 * kRec, a.rec2);
  bar_lds();
  SBP();

  // ---- 6: out = lrelu(IN2(y2) + shortcut)
  T* on = reinterpret_cast<T*>(a.out) + (long long)n * a.out_nstride + (long long)row0 * S;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = 4 * tid + q;
    if (e < 16 * S) {
      const int c = e / S, v = e - c * S;
      const float* r2 = rec + (32 + c) * kRec;
      float res = xres[q];
      if (sc) {
        const float* rr = rec + c * kRec;
        res = fmaf(rr[2], rt[c * SP + v] - rr[0], rr[3]);
      }
      st1(on + e, lrelu(fmaf(r2[2], yt[c * SP + v] - r2[0], r2[3]) + res));
    }
  }
  bar_lds();
  SBP();
#undef SBP
}

L3U_INLINE_HOST int device_cus() {   // compute units of the current device (cached)
  static int cache[64] = {0};
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  if (dev < 64 && cache[dev] > 0) return cache[dev];
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (dev < 64) cache[dev] = cus;
  return cus;
}

template <typename T>
int sblock_fwd_impl(const l3u_sblock_fwd_args* a, int N, int Cin, int Cout, int D, int H, int W,
                    hipStream_t stream) {
  L3U_REQUIRE(a != nullptr && N > 0);
  const int sc = a->w_sc != nullptr ? 1 : 0;
  const SbGeom g = sb_geom(Cin, Cout, D, H, W, sc);
  L3U_REQUIRE(g.ok && sb_blocks(N, Cout) <= device_cus());
  L3U_REQUIRE(a->x && a->w_dw1 && a->w_pw1 && a->g1 && a->b1 && a->w_dw2 && a->w_pw2 && a->g2 &&
              a->b2 && a->z1 && a->y1 && a->z2 && a->y2 && a->out && a->rec1 && a->rec2 && a->sync);
  L3U_REQUIRE(!sc || (a->r && a->g_sc && a->b_sc && a->rec_r));
  const bool v4 = g.S % 4 == 0 && a->x_nstride % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(a->x) % 16 == 0 && reinterpret_cast<uintptr_t>(a->z1) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(a->z2) % 16 == 0;
  if (v4)
    hipLaunchKernelGGL((sblock_fwd_kernel<T, 4>), dim3(sb_blocks(N, Cout)), dim3(kThreads), g.lds,
                       stream, *a, N, Cin, Cout, D, H, W, g.SP, g.ntile, g.P3, g.zrows, g.wreg);
  else
    hipLaunchKernelGGL((sblock_fwd_kernel<T, 1>), dim3(sb_blocks(N, Cout)), dim3(kThreads), g.lds,
                       stream, *a, N, Cin, Cout, D, H, W, g.SP, g.ntile, g.P3, g.zrows, g.wreg);
  L3U_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

int l3u_sblock_supported(int N, int Cin, int Cout, int D, int H, int W, int shortcut) {
  const SbGeom g = sb_geom(Cin, Cout, D, H, W, shortcut ? 1 : 0);
  return g.ok && N > 0 && sb_blocks(N, Cout) <= device_cus() ? 1 : 0;
}

int l3u_sblock_fwd(const l3u_sblock_fwd_args* a, int N, int Cin, int Cout, int D, int H, int W,
                   hipStream_t stream) {
  return sblock_fwd_impl<float>(a, N, Cin, Cout, D, H, W, stream);
}

int l3u_sblock_fwd_bf16(const l3u_sblock_fwd_args* a, int N, int Cin, int Cout, int D, int H, int W,
                        hipStream_t stream) {
  return sblock_fwd_impl<bf16>(a, N, Cin, Cout, D, H, W, stream);
}

}  // extern "C"
