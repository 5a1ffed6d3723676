// Channel-contraction GEMMs on the fp32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 fmac chain).
//   pw_fwd        Y[n][j][s] = sum_k Wm[j][k] X[n][k][s] (+bias[j]) (+Y)     (1x1x1 conv fwd / bwd-data,
//                 ConvTranspose3d(k2,s2) as a [Co*8 x Ci] GEMM)
//   pw_bwd_weight dW[j][k] = sum_{n,s} dY[n][j][s] X[n][k][s]                 (split-K partials)
// Replaces nn.Conv3d(Ci, Co, 1) of DepthwiseSeparableConv3d.pointwise (unet3d.py:18), the shortcut
// conv (unet3d.py:70-73), and the GEMM part of nn.ConvTranspose3d(Ci, Ci/2, 2, 2) (unet3d.py:119).
//
// Register-direct operand mapping (no LDS round trip for the streamed operand): the weights are
// the MFMA A operand (row i = output channel), X the B operand: a lane loads one float4
// X[k0 + (l>>4)][s + 4(l&15) .. +3] (each k-row of the wave is 256 contiguous bytes) and feeds
// component q to MFMA q, so MFMA q owns voxels {s + 4j + q}.  The accumulator of lane l then holds
// channels 4(l>>4) + r and the 4 CONSECUTIVE voxels 4(l&15) .. +3: a store instruction writes
// 64 consecutive voxels (256 B) per channel row.  Small K keeps the whole reduction in registers
// (weights read from L1/L2); larger K stages the weights per workgroup in LDS as Wt[k][j] (row
// stride padded to 16 mod 32 floats: conflict-free ds_read_b32 for the 2x16-lane groups).
// The pw_fwd epilogue can also emit per-(n, j) InstanceNorm partials (count, mean, M2) of its
// output tile (Chan merge later), so InstanceNorm statistics never re-read the activation.
#include "common.h"
using namespace l3u;

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

L3U_DEV f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// The streamed operand X[k][s .. s+3] (4 voxels, zero past S / past row K).  GATHER: X is the
// ConvTranspose3d(k2, s2) gradient read in place from the up-sampled tensor (its backward without
// a space-to-depth copy): row k = co*8 + (4a + 2b + c) at input voxel (z, y, x) is
// src[co][2z+a][2y+b][2x+c], channel stride 8S, dims (Dq, Hq, Wq) = the input (low-res) volume.
// With W % 4 == 0 the 4 voxels share an output row: two float4 loads of 8 consecutive floats and
// an even/odd pick.
template <bool VEC, bool GATHER, typename T>
L3U_DEV f4 load_x4(const T* __restrict__ xn, int kk, int K, int s, int lim, int S, int Hq,
                   int Wq) {   // voxels >= lim (<= S) read as zero
  f4 a = {0.f, 0.f, 0.f, 0.f};
  if (kk >= K) return a;
  if (GATHER) {
    const int a_ = (kk >> 2) & 1, b_ = (kk >> 1) & 1, c_ = kk & 1;
    const T* base = xn + (long long)(kk >> 3) * (8ll * S);
    if (VEC) {
      if (s < lim) {
        const int x = s % Wq, t = s / Wq, y = t % Hq, z = t / Hq;
        const T* p = base + ((long long)(2 * z + a_) * (2 * Hq) + (2 * y + b_)) * (2 * Wq) + 2 * x;
        const f4 lo = ldv4(p), hi = ldv4(p + 4);
        a = c_ ? f4{lo[1], lo[3], hi[1], hi[3]} : f4{lo[0], lo[2], hi[0], hi[2]};
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (s + q < lim) {
          const int x = (s + q) % Wq, t = (s + q) / Wq, y = t % Hq, z = t / Hq;
          a[q] = ld1(base + ((long long)(2 * z + a_) * (2 * Hq) + (2 * y + b_)) * (2 * Wq) + 2 * x + c_);
        }
    }
    return a;
  }
  const T* src = xn + (long long)kk * S + s;
  if (VEC) {
    if (s < lim) a = ldv4(src);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (s + q < lim) a[q] = ld1(src + q);
  }
  return a;
}

// ConvTranspose3d(k=2, s=2) epilogue: GEMM row j = co*8 + (4a + 2b + c) of input voxel s lands at
// out[co][2z+a][2y+b][2x+c] (+ bias[co]).  A lane holds rows j0 (c = 0) and j0 + 1 (c = 1) of the
// same 4 consecutive input voxels, i.e. 8 CONTIGUOUS outputs [2x0 .. 2x0+7]: two float4 stores.
// Requires W % 4 == 0 (VEC); otherwise per-voxel scalar stores.
template <bool VEC, typename T>
L3U_DEV void d2s_store2(T* outn, int j0, int Nout, const float* __restrict__ bias, int s, f4 v0,
                        f4 v1, int S, int D, int H, int W) {
  const bool ok = j0 < Nout;
  const int co = j0 >> 3, a = (j0 >> 2) & 1, bq = (j0 >> 1) & 1;
  const float bv = (bias && ok) ? bias[co] : 0.f;
  v0 += bv;
  v1 += bv;
  T* oc = outn + (long long)co * (8ll * S);
  if (VEC) {
    if (ok && s < S) {
      const int x = s % W, t = s / W, y = t % H, z = t / H;
      T* dst = oc + ((long long)(2 * z + a) * (2 * H) + (2 * y + bq)) * (2 * W) + 2 * x;
      stv4(dst, f4{v0[0], v1[0], v0[1], v1[1]});
      stv4(dst + 4, f4{v0[2], v1[2], v0[3], v1[3]});
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (ok && s + q < S) {
        const int x = (s + q) % W, t = (s + q) / W, y = t % H, z = t / H;
        T* dst = oc + ((long long)(2 * z + a) * (2 * H) + (2 * y + bq)) * (2 * W) + 2 * x;
        st1(dst, v0[q]);
        st1(dst + 1, v1[q]);
      }
    }
  }
}

// KS > 0: the whole reduction (K <= 4*KS) in registers, X and weight loads (weights straight
// from L1/L2, no LDS staging barrier) all issued before the first MFMA; KS = 0: generic K loop
// with the weights staged through LDS in chunks of 128 reduction rows.
template <typename T, int NC, int NSW, bool VEC, int XM, int KS>   // XM: 0 plain, 1 scatter epilogue, 2 gathered X
__global__ __launch_bounds__(256) void pw_fwd_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w, int wl,
    const float* __restrict__ bias, T* __restrict__ y, long long yns, int accumulate,
    float* __restrict__ stat_part, int K, int Nout, int S, int nsb, int Dq, int Hq, int Wq,
    const T* __restrict__ x2 = nullptr, long long xns2 = 0, const float* __restrict__ w2 = nullptr,
    T* __restrict__ y2 = nullptr, long long yns2 = 0, float* __restrict__ stat2 = nullptr,
    int N1 = 0) {
  L3U_STAMP_SCOPE(101);
  kargs_now(x, xns, w, wl, bias, y, yns, accumulate, stat_part, K, Nout, S, nsb, Dq, Hq, Wq, x2, xns2,
            w2, y2, yns2, stat2, N1);
  constexpr int CO_BLK = 16 * NC;
  constexpr int TSB = 256 * NSW;
  constexpr int WS = (CO_BLK % 32 == 16) ? CO_BLK : CO_BLK + 16;
  constexpr int KCH = 128;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int sb = blockIdx.x, co0 = blockIdx.y * CO_BLK;
  int n = blockIdx.z;
  if (x2 != nullptr && n >= N1) {   // the second problem of a paired launch (l3u_pw_fwd2)
    n -= N1; x = x2; xns = xns2; w = w2; y = y2; yns = yns2; stat_part = stat2;
  }
  const int Kp = (K + 3) & ~3;
  const int wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const T* xn = x + (long long)n * xns;
  const int sbase = sb * TSB + wave * 64 * NSW;

  f4 acc[NSW][NC][4];
#pragma unroll
  for (int j = 0; j < NSW; ++j)
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[j][m][q] = f4{0.f, 0.f, 0.f, 0.f};

  if constexpr (KS > 0) {
    f4 a[KS][NSW];
    float b[KS][NC];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kk = 4 * ks + lk;
#pragma unroll
      for (int j = 0; j < NSW; ++j) {
        a[ks][j] = load_x4<VEC, XM == 2>(xn, kk, K, sbase + j * 64 + 4 * lr, S, S, Hq, Wq);
      }
#pragma unroll
      for (int m = 0; m < NC; ++m) {
        const int co = co0 + 16 * m + lr;
        b[ks][m] = (kk < K && co < Nout) ? (wl == 0 ? w[(long long)co * K + kk] : w[(long long)kk * Nout + co]) : 0.f;
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NSW; ++j)
#pragma unroll
        for (int m = 0; m < NC; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[j][m][q] = mfma4(b[ks][m], a[ks][j][q], acc[j][m][q]);
  } else {
  // the weight operand is staged through LDS in chunks of KCH reduction rows
  for (int kc0 = 0; kc0 < Kp; kc0 += KCH) {
  const int kc1 = min(Kp, kc0 + KCH);
  if (kc0 > 0) __syncthreads();
  for (int i = tid; i < (kc1 - kc0) * CO_BLK; i += 256) {
    const int kr = i / CO_BLK, j = i - kr * CO_BLK, k = kc0 + kr, co = co0 + j;
    float v = 0.f;
    if (k < K && co < Nout) v = wl == 0 ? w[(long long)co * K + k] : w[(long long)k * Nout + co];
    lds[kr * WS + j] = v;
  }
  __syncthreads();
#pragma unroll 8
  for (int k0 = kc0; k0 < kc1; k0 += 4) {
    const int kk = k0 + lk;
    f4 a[NSW];
#pragma unroll
    for (int j = 0; j < NSW; ++j) {
      a[j] = load_x4<VEC, XM == 2>(xn, kk, K, sbase + j * 64 + 4 * lr, S, S, Hq, Wq);
    }
    float b[NC];
#pragma unroll
    for (int m = 0; m < NC; ++m) b[m] = lds[(kk - kc0) * WS + 16 * m + lr];
#pragma unroll
    for (int j = 0; j < NSW; ++j)
#pragma unroll
      for (int m = 0; m < NC; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[j][m][q] = mfma4(b[m], a[j][q], acc[j][m][q]);
  }
  }
  }

  // epilogue: lane (lr, lk) holds Y[co0 + 16m + 4lk + r][sbase + 64j + 4lr + q]: per (m, r) the
  // 16 lanes of a row store 64 consecutive voxels of one channel (256 B, coalesced)
  T* yn = y + (long long)n * yns;
  if (XM == 1) {
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int j = 0; j < NSW; ++j)
#pragma unroll
        for (int rp = 0; rp < 4; rp += 2)
          d2s_store2<VEC>(yn, co0 + 16 * m + 4 * lk + rp, Nout, bias, sbase + j * 64 + 4 * lr,
                          f4{acc[j][m][0][rp], acc[j][m][1][rp], acc[j][m][2][rp], acc[j][m][3][rp]},
                          f4{acc[j][m][0][rp + 1], acc[j][m][1][rp + 1], acc[j][m][2][rp + 1],
                             acc[j][m][3][rp + 1]},
                          S, Dq, Hq, Wq);
    return;
  }
  float lsum[NC][4];
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * m + 4 * lk + r;
      const bool cok = co < Nout;
      const float bv = (bias && cok) ? bias[co] : 0.f;
      lsum[m][r] = 0.f;
#pragma unroll
      for (int j = 0; j < NSW; ++j) {
        const int s = sbase + j * 64 + 4 * lr;
        f4 v = f4{acc[j][m][0][r], acc[j][m][1][r], acc[j][m][2][r], acc[j][m][3][r]} + bv;
        T* dst = yn + (long long)co * S + s;
        if (cok) {
          if (VEC) {
            if (s < S) {
              if (accumulate) v += ldv4(dst);
              stv4(dst, v);
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (s + q < S) {
                if (accumulate) v[q] += ld1(dst + q);
                st1(dst + q, v[q]);
              }
          }
        }
        v = round_to(v, dst);   // statistics of the stored values
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[j][m][q][r] = v[q];                       // keep the stored value for the stats
          if (s + q < S) lsum[m][r] += v[q];
        }
      }
    }
  if (stat_part == nullptr) return;
  // per-channel block statistics (two-pass within the tile: mean, then M2 about that mean):
  // row sums over the 16 voxel lanes by DPP, then the 4 waves through LDS in fixed order
  float* red = lds;                                     // [4][CO_BLK] (weights no longer needed)
  const int s_lo = sb * TSB;
  const int cnt = min(TSB, S - s_lo);
  __syncthreads();
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = row_sum16(lsum[m][r]);
      if (lr == 0) red[wave * CO_BLK + 16 * m + 4 * lk + r] = v;
    }
  __syncthreads();
  float mean[NC][4];
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int jj = 16 * m + 4 * lk + r;
      mean[m][r] = ((red[jj] + red[CO_BLK + jj]) + (red[2 * CO_BLK + jj] + red[3 * CO_BLK + jj])) / (float)cnt;
    }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < NSW; ++j) {
        const int s = sbase + j * 64 + 4 * lr;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (s + q < S) {
            const float d = acc[j][m][q][r] - mean[m][r];
            v = fmaf(d, d, v);
          }
      }
      v = row_sum16(v);
      if (lr == 0) red[wave * CO_BLK + 16 * m + 4 * lk + r] = v;
    }
  __syncthreads();
  if (wave == 0 && lr == 0) {
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jj = 16 * m + 4 * lk + r, co = co0 + jj;
        if (co < Nout) {
          const float m2 = (red[jj] + red[CO_BLK + jj]) + (red[2 * CO_BLK + jj] + red[3 * CO_BLK + jj]);
          float* o = stat_part + (((long long)n * Nout + co) * nsb + sb) * 3;
          o[0] = (float)cnt;
          o[1] = mean[m][r];
          o[2] = m2;
        }
      }
  }
}

// Small-volume variant (per-sample S < 8192: the 12^3 / 6^3 levels): the 4 waves of a workgroup
// share ONE 64-voxel tile and split the reduction dimension K (k-steps interleaved by wave), then
// combine through LDS in a fixed order; weights are read straight from L2 (they are tiny and
// every workgroup re-reads them).  This turns an 8-workgroup grid into hundreds.
template <typename T, int NC, bool VEC, int XM, int KSM>
__global__ __launch_bounds__(256) void pw_fwd_ks_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w, int wl,
    const float* __restrict__ bias, T* __restrict__ y, long long yns, int accumulate,
    float* __restrict__ stat_part, int K, int Nout, int S, int nsb, int Dq, int Hq, int Wq,
    const T* __restrict__ x2 = nullptr, long long xns2 = 0, const float* __restrict__ w2 = nullptr,
    T* __restrict__ y2 = nullptr, long long yns2 = 0, float* __restrict__ stat2 = nullptr,
    int N1 = 0) {
  L3U_STAMP_SCOPE(102);
  kargs_now(x, xns, w, wl, bias, y, yns, accumulate, stat_part, K, Nout, S, nsb, Dq, Hq, Wq, x2, xns2,
            w2, y2, yns2, stat2, N1);
  constexpr int CO_BLK = 16 * NC;
  constexpr int NT = NC * 16;   // accumulator floats per lane
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [4 waves][NT][64 lanes]
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int sb = blockIdx.x, co0 = blockIdx.y * CO_BLK;
  int n = blockIdx.z;
  if (x2 != nullptr && n >= N1) {   // the second problem of a paired launch (l3u_pw_fwd2)
    n -= N1; x = x2; xns = xns2; w = w2; y = y2; yns = yns2; stat_part = stat2;
  }
  const T* xn = x + (long long)n * xns;
  const int s = sb * 64 + 4 * lr;
  const int ksteps = (K + 3) >> 2;
  f4 acc[NC][4];
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = f4{0.f, 0.f, 0.f, 0.f};
  // KSM k-steps per wave in flight: every load of a round is issued before its first MFMA (one
  // memory round trip per round); 8 for latency-bound grids, 4 keeps the registers of big ones
  for (int k0s = wave; k0s < ksteps; k0s += 4 * KSM) {
    f4 av[KSM];
    float bv[KSM][NC];
#pragma unroll
    for (int u = 0; u < KSM; ++u) {
      const int kk = 4 * (k0s + 4 * u) + lk;
      av[u] = load_x4<VEC, XM == 2>(xn, kk, K, s, S, S, Hq, Wq);
#pragma unroll
      for (int m = 0; m < NC; ++m) {
        const int co = co0 + 16 * m + lr;
        bv[u][m] = 0.f;
        if (kk < K && co < Nout) bv[u][m] = wl == 0 ? w[(long long)co * K + kk] : w[(long long)kk * Nout + co];
      }
    }
#pragma unroll
    for (int u = 0; u < KSM; ++u)
      if (k0s + 4 * u < ksteps) {
#pragma unroll
        for (int m = 0; m < NC; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[m][q] = mfma4(bv[u][m], av[u][q], acc[m][q]);
      }
  }
  // cross-wave combine through LDS, value-major ([wave][value][lane]: consecutive lanes hit
  // consecutive banks, conflict-free).  Every wave parks its partials; wave w then owns output
  // tile m = w (16 channels x 64 voxels) and adds the four waves' partials of that tile in wave
  // order (fixed: deterministic), so the epilogue stores are spread over min(NC, 4) waves.
#ifdef L3U_STAMP_KS
  L3U_STAMP_MARK(0);   // stamp variant: the k-loop (loads + MFMAs) done
#endif
  {
    float* dst = lds + wave * NT * 64 + l;
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[((m * 4 + q) * 4 + r) * 64] = acc[m][q][r];
  }
  __syncthreads();
#ifndef L3U_STAMP_KS
  L3U_STAMP_MARK(0);
#endif
  const int m = wave;
  if (m >= NC) return;
  f4 t4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* src = lds + ((m * 4 + q) * 4 + r) * 64 + l;
      t4[q][r] = ((src[0] + src[NT * 64]) + src[2 * NT * 64]) + src[3 * NT * 64];
    }
  }
  L3U_STAMP_MARK(1);
  // epilogue: lane (lr, lk) holds Y[co0 + 16m + 4lk + r][sb*64 + 4lr + q]
  T* yn = y + (long long)n * yns;
  const int sv = sb * 64 + 4 * lr;
  if (XM == 1) {
#pragma unroll
    for (int rp = 0; rp < 4; rp += 2)
      d2s_store2<VEC>(yn, co0 + 16 * m + 4 * lk + rp, Nout, bias, sv,
                      f4{t4[0][rp], t4[1][rp], t4[2][rp], t4[3][rp]},
                      f4{t4[0][rp + 1], t4[1][rp + 1], t4[2][rp + 1], t4[3][rp + 1]}, S, Dq, Hq, Wq);
    return;
  }
  const int cnt = min(64, S - sb * 64);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + 16 * m + 4 * lk + r;
    const bool cok = co < Nout;
    const float bv = (bias && cok) ? bias[co] : 0.f;
    f4 v = f4{t4[0][r], t4[1][r], t4[2][r], t4[3][r]} + bv;
    T* dst = yn + (long long)co * S + sv;
    if (cok) {
      if (VEC) {
        if (sv < S) {
          if (accumulate) v += ldv4(dst);
          stv4(dst, v);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (sv + q < S) {
            if (accumulate) v[q] += ld1(dst + q);
            st1(dst + q, v[q]);
          }
      }
    }
    v = round_to(v, dst);   // statistics of the stored values
    if (stat_part != nullptr) {
      float ls = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (sv + q < S) ls += v[q];
      const float mean = row_sum16(ls) / (float)cnt;
      float m2 = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (sv + q < S) {
          const float d = v[q] - mean;
          m2 = fmaf(d, d, m2);
        }
      m2 = row_sum16(m2);
      if (lr == 0 && cok) {
        float* o = stat_part + (((long long)n * Nout + co) * nsb + sb) * 3;
        o[0] = (float)cnt;
        o[1] = mean;
        o[2] = m2;
      }
    }
  }
}

// One-wave form for the mid-size levels (4096 <= S < 32768: 24^3) with K <= 64: a 64-thread
// workgroup owns one 64-voxel tile x 16 NC output channels and runs the WHOLE reduction in
// registers (K / 4 float4 loads of X in flight, then K / 4 * 4 * NC MFMAs in one chain per
// accumulator, the pw_fwd k order), so there is no cross-wave LDS combine and no 32 KB LDS
// tile per workgroup (pw_fwd_ks at 24^3: four waves of one k-step each, five workgroups per CU,
// two rounds of waves).  Same epilogue and (count, mean, M2) partials per 64-voxel tile as
// pw_fwd_ks (l3u_pw_stat_nsb is unchanged).
template <typename T, int NC, int KS>
__global__ __launch_bounds__(64) void pw_fwd_w1_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w, int wl,
    const float* __restrict__ bias, T* __restrict__ y, long long yns, int accumulate,
    float* __restrict__ stat_part, int K, int Nout, int S, int nsb,
    const T* __restrict__ x2, long long xns2, const float* __restrict__ w2, T* __restrict__ y2,
    long long yns2, float* __restrict__ stat2, int N1) {
  L3U_STAMP_SCOPE(110);
  kargs_now(x, xns, w, wl, bias, y, yns, accumulate, stat_part, K, Nout, S, nsb, x2, xns2, w2, y2,
            yns2, stat2, N1);
  const int l = threadIdx.x, lr = l & 15, lk = l >> 4;
  const int sb = blockIdx.x, co0 = blockIdx.y * 16 * NC;
  int n = blockIdx.z;
  if (x2 != nullptr && n >= N1) {   // the second problem of a paired launch (l3u_pw_fwd2)
    n -= N1; x = x2; xns = xns2; w = w2; y = y2; yns = yns2; stat_part = stat2;
  }
  const T* xn = x + (long long)n * xns;
  const int sv = sb * 64 + 4 * lr;
  f4 a[KS];
  float b[KS][NC];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int kk = 4 * ks + lk;
    a[ks] = load_x4<true, false>(xn, kk, K, sv, S, S, 0, 0);
#pragma unroll
    for (int m = 0; m < NC; ++m) {
      const int co = co0 + 16 * m + lr;
      b[ks][m] = (kk < K && co < Nout) ? (wl == 0 ? w[(long long)co * K + kk] : w[(long long)kk * Nout + co]) : 0.f;
    }
  }
  f4 acc[NC][4];
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[m][q] = mfma4(b[ks][m], a[ks][q], acc[m][q]);
  // epilogue: lane (lr, lk) holds Y[co0 + 16m + 4lk + r][sb*64 + 4lr + q]
  T* yn = y + (long long)n * yns;
  const int cnt = min(64, S - sb * 64);
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * m + 4 * lk + r;
      const bool cok = co < Nout;
      const float bv = (bias && cok) ? bias[co] : 0.f;
      f4 v = f4{acc[m][0][r], acc[m][1][r], acc[m][2][r], acc[m][3][r]} + bv;
      T* dst = yn + (long long)co * S + sv;
      if (cok && sv < S) {
        if (accumulate) v += ldv4(dst);
        stv4(dst, v);
      }
      v = round_to(v, dst);   // statistics of the stored values
      if (stat_part != nullptr) {
        float ls = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (sv + q < S) ls += v[q];
        const float mean = row_sum16(ls) / (float)cnt;
        float m2 = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (sv + q < S) {
            const float d = v[q] - mean;
            m2 = fmaf(d, d, m2);
          }
        m2 = row_sum16(m2);
        if (lr == 0 && cok) {
          float* o = stat_part + (((long long)n * Nout + co) * nsb + sb) * 3;
          o[0] = (float)cnt;
          o[1] = mean;
          o[2] = m2;
        }
      }
    }
}

// dW[j][k] partial over one voxel chunk of one sample.  A = dY (rows j), B = X^T (cols k),
// the MFMA k-dimension is the voxel: lane l loads float4 dY[j0+16mo+(l&15)][s+4(l>>4)..+3] and
// X[k0+16mi+(l&15)][s+4(l>>4)..+3]; component q feeds MFMA q.
template <typename TD, typename TX, int NJ, int NK, bool VEC, bool GATHER>
__global__ __launch_bounds__(256) void pw_bwd_weight_kernel(
    const TD* __restrict__ dy, long long dyns, const TX* __restrict__ x, long long xns,
    float* __restrict__ part, float* __restrict__ bsum, int J, int K, int S, int SCH, int nsc,
    int Hq, int Wq) {
  L3U_STAMP_SCOPE(103);
  constexpr int TJ = 16 * NJ, TK = 16 * NK;
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [64][T]
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int sc = blockIdx.x % nsc, n = blockIdx.x / nsc;
  const int ntk = (K + TK - 1) / TK;
  const int j0 = (blockIdx.y / ntk) * TJ, k0 = (blockIdx.y % ntk) * TK;
  const TD* dyn = dy + (long long)n * dyns;
  const TX* xn = x + (long long)n * xns;
  const int s_lo = sc * SCH, s_hi = min(S, s_lo + SCH);

  f4 acc[NJ][NK];
#pragma unroll
  for (int a = 0; a < NJ; ++a)
#pragma unroll
    for (int b = 0; b < NK; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  // bsum (GATHER, the ConvTranspose3d bias): row sums of the X operand over the chunk, by the
  // workgroups of the first J tile
  const bool do_b = GATHER && bsum != nullptr && j0 == 0;
  float bacc[NK];
#pragma unroll
  for (int b = 0; b < NK; ++b) bacc[b] = 0.f;

#pragma unroll 4
  for (int s = s_lo + wave * 16; s < s_hi; s += 64) {
    const int sl = s + 4 * lk;
    f4 av[NJ], bv[NK];
#pragma unroll
    for (int a = 0; a < NJ; ++a) {
      const int jj = j0 + 16 * a + lr;
      av[a] = f4{0.f, 0.f, 0.f, 0.f};
      if (jj < J) {
        const TD* src = dyn + (long long)jj * S + sl;
        if (VEC) {
          if (sl < s_hi) av[a] = ldv4(src);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (sl + q < s_hi) av[a][q] = ld1(src + q);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NK; ++b)
      bv[b] = load_x4<VEC, GATHER>(xn, k0 + 16 * b + lr, K, sl, s_hi, S, Hq, Wq);
    if (do_b) {
#pragma unroll
      for (int b = 0; b < NK; ++b) bacc[b] += (bv[b][0] + bv[b][1]) + (bv[b][2] + bv[b][3]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int a = 0; a < NJ; ++a)
#pragma unroll
        for (int b = 0; b < NK; ++b) acc[a][b] = mfma4(av[a][q], bv[b][q], acc[a][b]);
  }
  // fixed-order cross-wave reduction through LDS (value-major [value][lane]: conflict-free)
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int a = 0; a < NJ; ++a)
#pragma unroll
        for (int b = 0; b < NK; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int idx = ((a * NK + b) * 4 + r) * 64 + l;
            lds[idx] = wv == 0 ? acc[a][b][r] : lds[idx] + acc[a][b][r];
          }
    }
    __syncthreads();
  }
  if (wave == 0) {
    float* o = part + (long long)blockIdx.x * J * K;
#pragma unroll
    for (int a = 0; a < NJ; ++a)
#pragma unroll
      for (int b = 0; b < NK; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int jj = j0 + 16 * a + 4 * lk + r, kk = k0 + 16 * b + lr;
          if (jj < J && kk < K) o[(long long)jj * K + kk] = lds[((a * NK + b) * 4 + r) * 64 + l];
        }
  }
  if (do_b) {   // block-uniform: rows over the lanes lk, then the waves in order, then co = k/8
    __syncthreads();
    float* bl = lds;                                  // [4 waves][16 * NK]
#pragma unroll
    for (int b = 0; b < NK; ++b) {
      float v = bacc[b];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lk == 0) bl[wave * 16 * NK + 16 * b + lr] = v;
    }
    __syncthreads();
    if (tid < 2 * NK) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = 8 * tid + i;
        v += ((bl[row] + bl[16 * NK + row]) + bl[32 * NK + row]) + bl[48 * NK + row];
      }
      const int co = (k0 >> 3) + tid;
      if (8 * co < K) bsum[(long long)(blockIdx.x) * (K / 8) + co] = v;
    }
  }
}

// Fused backward of a 1x1 conv Y = W X (W [J][K]) for J <= 32, K <= 64 (the 48^3 / 24^3 levels):
// one pass over a voxel chunk (one wave per 64 voxels, up to 8 waves: a chunk is one sweep) reads
// dY once per 16*NK columns of K (grid.y splits K for parallelism; dY re-reads hit L2) and
// produces both
//   dX[k][s]  = sum_j W[j][k] dY[j][s]              (data gradient, optional accumulate)
//   part[j][k] = sum_{s in chunk} dY[j][s] X[k][s]  (weight-gradient partial, fixed order)
// PRO 1 forms dY on the fly from the InstanceNorm backward of the preceding norm
// (in_bwd_apply: dY = f*(dpre - M1 - (y - mu)*rs*M2), same float expression), so that tensor
// is never written.  Per wave and 64-voxel tile: dY is loaded in the data-gradient B layout
// (row 4jr + lk, voxels 4lr..+3) and feeds its MFMAs straight from registers; a copy goes to a
// wave-private LDS tile (row stride 68 floats) from which the weight-gradient A operand
// (row lr, voxels 16g + 4lk..+3) is read back transposed, conflict-free.  X is only needed by
// the weight gradient and is loaded in its B layout.  The weights sit in LDS as W[j][k] with a
// row stride = 16 mod 64 floats (conflict-free A-operand reads for the data gradient).
// the second problem of a paired block-tail launch (l3u_pw_bwd_tail_pair, PRO 2): the same
// block tail (dout, out, tail partials) for the other pointwise backward of the block
// (conv2.pointwise, sel 1, or the shortcut, sel 2); blockIdx.z == 1
#ifndef L3U_DYT_SWZ
#define L3U_DYT_SWZ 1
#endif
constexpr bool kDyTileSwz = L3U_DYT_SWZ != 0;
constexpr int kDyTileDS = kDyTileSwz ? 64 : 68;   // dY tile row stride (floats)
// float offset of quad q (4 voxels) of row r in a wave's dY tile
L3U_DEV int dyt_at(int r, int q) {
  return r * kDyTileDS + 4 * (kDyTileSwz ? (q ^ (r & 15)) : q);
}

template <typename T>
struct TailSecond {
  const T* yr; long long yrns; const float* rec; const T* x; long long xns; const float* w;
  float* dx; long long dxns; int accumulate; float* part; int K; int sel;
};

#ifndef L3U_PWBF_WAVES1
#define L3U_PWBF_WAVES1 4
#endif
// minimum waves per SIMD asked of the 16-row forms with up to 32 columns (0: the compiler's
// choice, 4 for the block-tail forms at 106-108 VGPRs)
constexpr int kPwbfWaves1 = L3U_PWBF_WAVES1;
#ifndef L3U_PWBF_PB
#define L3U_PWBF_PB 4
#endif
constexpr int kPwbfPB = L3U_PWBF_PB;
#ifndef L3U_PWBF_WAVES2
#define L3U_PWBF_WAVES2 4
#endif
// ... and of the 32-row forms without a prologue and with up to 32 columns (184 -> 88 / 112
// VGPRs, no spill; the prologue forms spill 11-38 VGPRs at 4 waves)
constexpr int kPwbfWaves2 = L3U_PWBF_WAVES2;
#ifndef L3U_PWBF_WAVES1K1
#define L3U_PWBF_WAVES1K1 5
#endif
// ... and of the 16-row, 16-column forms (80 VGPRs at 6 waves without a spill; the 32-column ones
// spill 11-20 there)
constexpr int kPwbfWaves1k1 = L3U_PWBF_WAVES1K1;
#ifndef L3U_PWBF_WAVES3
#define L3U_PWBF_WAVES3 3
#endif
// ... and of the 32-row forms with a prologue (0: the compiler's choice)
constexpr int kPwbfWaves3 = L3U_PWBF_WAVES3;
template <int NJ, int NK, int PRO>
constexpr int pwbf_waves() {
  return NJ == 1 ? (NK == 1 && kPwbfWaves1k1 > 0 ? kPwbfWaves1k1
                                                 : (NK <= 2 && kPwbfWaves1 > 0 ? kPwbfWaves1 : 1))
                 : (PRO == 0 && NK <= 2 && kPwbfWaves2 > 0 ? kPwbfWaves2
                                                           : (PRO && kPwbfWaves3 > 0 ? kPwbfWaves3 : 1));
}
template <typename T, int NJ, int NK, int PRO, bool R1 = false, bool R1B = false, bool PL = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(pwbf_waves<NJ, NK, PRO>()))) void pw_bwd_fused_kernel(
    const float* __restrict__ dy, long long dyns, const T* __restrict__ yin, long long yns,
    const float* __restrict__ rec, const double* __restrict__ in_part, int npart,
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    float* __restrict__ dx, long long dxns, int accumulate, float* __restrict__ part, int N, int J,
    int K, int S, int SCH, int nsc, const T* __restrict__ oin = nullptr, long long oins = 0,
    int sel = 1, const float* __restrict__ dscale = nullptr, const float* __restrict__ dpool = nullptr,
    long long dpns = 0, const unsigned char* __restrict__ pidx = nullptr, int Hf = 0, int Wf = 0,
    TailSecond<T> p2 = TailSecond<T>{}) {
  L3U_STAMP_SCOPE(104);
  constexpr int TJ = 16 * NJ, TK = 16 * NK, JR = TJ / 4;
  if (PRO == 2 && blockIdx.z == 1) {   // paired tail launch, second problem
    yin = p2.yr; yns = p2.yrns; rec = p2.rec; x = p2.x; xns = p2.xns; w = p2.w; dx = p2.dx;
    dxns = p2.dxns; accumulate = p2.accumulate; part = p2.part; K = p2.K; sel = p2.sel;
  }
  if ((int)blockIdx.y * TK >= K) return;   // the narrower problem's unused column blocks
  constexpr int WS = TK + ((16 - TK) % 64 + 64) % 64;   // >= TK, = 16 mod 64
  // dY tile: row stride DS floats; with kDyTileSwz the 16 quads of a row are XOR-swizzled by the
  // row (quad q of row r at q ^ (r & 15)): the b128 writes (8 lanes of one row) and the
  // transposed b128 reads (lane (lr, lk) reads quad 4 gg + lk of row lr; gfx950 serves a
  // ds_read_b128 in 4 lane groups of 16) are both bank-conflict-free.  The unswizzled stride-68
  // image had a 2-way conflict in every read group (round-4 SQ pass: 404k conflict cycles per
  // 553k LDS instructions in the 48^3 tail pair)
  constexpr int DS = kDyTileDS;
  constexpr int PS = 8;                                 // lanes per channel for the IN sums
  static_assert(NJ == 2 || NK * 256 <= 16 * DS, "weight-gradient reduction must fit in the dY tiles");
  __shared__ __attribute__((aligned(16))) float w_l[TJ * WS];
  __shared__ __attribute__((aligned(16))) float coef[PRO ? TJ * 8 : 1];
  __shared__ double psum[PRO ? TJ * PS * 2 : 1];
  // the waves' dY tiles, sized by the launch for the block's wave count (a static [8] array held
  // 70 KB at TJ = 32 for 4-wave blocks: two workgroups per CU instead of four)
  extern __shared__ __attribute__((aligned(16))) float dyt_lds[];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int nthr = blockDim.x, nwv = nthr >> 6;         // one sweep: SCH == 64 * nwv
  const int sc = blockIdx.x % nsc, n = blockIdx.x / nsc, k0 = blockIdx.y * TK;
  const int s_lo = sc * SCH, s_hi = min(S, s_lo + SCH);
  const int sw = s_lo + 64 * wave;
  const int sd = sw + 4 * lr;                           // data-gradient layout voxels
  const float* dyn = dy + (long long)n * dyns;
  const T* xn = x + (long long)n * xns;
  float* dxn = dx + (long long)n * dxns;

  // 0. the small per-workgroup operands are requested FIRST, into registers: the weight slice,
  // (PRO) the first batch of the InstanceNorm-backward partials and the records.  Vector loads
  // complete in order, so operands requested behind the streamed tile could only be consumed once
  // the whole tile had arrived: the weight staging loop and the partial batch were two more
  // dependent round trips, and the records a third behind the first barrier (round 6 ISA
  // review).  Requested first, the partial sums, the barrier and the coefficients overlap the
  // tile's flight.  Clamped unconditional loads (nthr >= 256: pw_chunk_ok), selected at use.
  constexpr int PB = NJ == 1 && NK == 1 && kPwbfWaves1k1 >= 6 ? 2 : kPwbfPB;   // partials per batch
  // (the 16-column forms at 6 waves per SIMD have no room for the early batch: 80 VGPRs, 8-10
  // spilled; they request it behind the tile as before)
  constexpr bool EP = PRO && !(NJ == 1 && NK == 1 && kPwbfWaves1k1 >= 6) && !PL;   // (PL: its pool loads)
  constexpr int WPT = (TJ * WS + 255) / 256;
  float wreg[WPT];
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int i = min(tid + u * nthr, TJ * WS - 1), j = i / WS, kc = i - j * WS;
    wreg[u] = w[(long long)min(j, J - 1) * K + min(k0 + kc, K - 1)];
  }
  const int pj = min(tid / PS, J - 1), psub = tid % PS;
  const int pst = PRO == 2 ? 3 : 2, po1 = PRO == 2 ? sel : 1;
  const double* pp = in_part + ((long long)pj * N + n) * npart * pst;
  double pa0[EP ? PB : 1], pa1[EP ? PB : 1];
  float q0 = 0.f, q1 = 0.f, q5 = 0.f, q7 = 0.f;
  if constexpr (EP) {
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int i = min(psub + u * PS, npart - 1);
      pa0[u] = pp[i * pst];
      pa1[u] = pp[i * pst + po1];
    }
  }
  if constexpr (PRO) {
    const float* q = rec + ((long long)n * J + min(tid, J - 1)) * kRec;
    q0 = q[0]; q1 = q[1]; q5 = q[5]; q7 = q[7];
  }

  // rank-1 dout[j] = dscale[j] * dz (l3u_outconv_bwd_dz): the scales are small operands too
  float dsv[PRO == 2 && !PL ? JR : 1];   // (never with the pool fold: encoder blocks)
  if constexpr (PRO == 2 && !PL) {
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) dsv[jr] = dscale != nullptr ? dscale[min(4 * jr + lk, J - 1)] : 1.f;
  }

  // 1. then every streamed load of the tile, unconditional at clamped addresses and zeroed after
  // the load where it lies outside the tile: a branch around a load leaves the wait-count pass
  // unsure how many loads follow the small operands, and it then waits for the whole tile before
  // the coefficients
  const bool sok = sd < s_hi;
  const int sdc = sok ? sd : s_hi - 4;
  const long long gst = (PRO == 2 && dscale != nullptr) ? 0ll : (long long)S;   // rank-1 dz: one row
  f4 g[JR], yv[PRO ? JR : 1], ov[PRO == 2 ? JR : 1];
  // PL (PRO 2): + the next level's MaxPool3d backward (folded; a template flag so that the other
  // forms carry no pool code), the pooled gradient and argmax loads unconditional as well
  int pz = 0, py = 0, px = 0;
  if constexpr (PL) {
    const int HW = Hf * Wf;
    pz = fdiv(sdc, HW, 1.f / HW);
    const int rm = sdc - pz * HW;
    py = fdiv(rm, Wf, 1.f / Wf);
    px = rm - py * Wf;
  }
#pragma unroll
  for (int jr = 0; jr < JR; ++jr) {
    const int jc = min(4 * jr + lk, J - 1);
    g[jr] = ldv4(dyn + (long long)jc * gst + sdc);
    if constexpr (PL)
      g[jr] = unpool_add(g[jr], dpool + (long long)n * dpns + (long long)jc * (S / 8),
                         pidx + ((long long)n * J + jc) * (S / 8), pz, py, px, Hf, Wf);
  }
  if (PRO == 2) {   // the block output (LeakyReLU mask of the tail)
    const T* on = oin + (long long)n * oins;
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) ov[jr] = ldv4(on + (long long)min(4 * jr + lk, J - 1) * S + sdc);
  }
  // R1 (yns < 0): a rank-1 normalised operand, channel j = rec[j][7] * one stored channel
  // (include/l3u.h); a template flag so that the other variants keep their registers.  R1B: only
  // the paired launch's second problem (the first block's shortcut) has the rank-1 operand
  const bool yk = R1B ? (PRO == 2 && blockIdx.z == 1) : (PRO && R1);
  if (PRO) {
    const T* yn = yin + (long long)n * (yk ? -yns : yns);
#pragma unroll
    for (int jr = 0; jr < JR; ++jr)
      yv[jr] = ldv4(yn + (yk ? 0ll : (long long)min(4 * jr + lk, J - 1) * S) + sdc);
  }
#pragma unroll
  for (int jr = 0; jr < JR; ++jr) {
    const bool ok = 4 * jr + lk < J && sok;
    if constexpr (PRO == 2 && !PL) g[jr] = dsv[jr] * g[jr];   // (dsv = 1 without dscale: exact)
    const f4 z4 = {0.f, 0.f, 0.f, 0.f};
    g[jr] = ok ? g[jr] : z4;
    if (PRO == 2) ov[jr] = ok ? ov[jr] : z4;
    if (PRO) yv[jr] = ok ? yv[jr] : z4;
  }
  // X (the weight gradient's B operand): with a prologue (PRO 1 / 2) it is requested after dY is
  // formed, so that the dY / out / y registers are dead by then (TJ = 32, TK = 64: 226 -> 166
  // VGPRs, 2 -> 3 waves per SIMD; TJ = 16: 4 -> 5 for the IN-prologue forms) and its loads
  // overlap the data-gradient MFMAs and stores (config 5 -175 us, 48^3 -18 us); PRO 0 first
  constexpr bool XL = PRO == 0;
  f4 xv[4][NK];
  auto load_xv = [&] {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg)
#pragma unroll
      for (int b = 0; b < NK; ++b)
        xv[gg][b] = load_x4<true, false>(xn, k0 + 16 * b + lr, K, sw + 16 * gg + 4 * lk, s_hi, S, 0, 0);
  };
  if constexpr (XL) load_xv();

  // 2. the weight slice into LDS and (PRO) the per-channel InstanceNorm-backward coefficients,
  // whose fp64 partial sums are spread over PS lanes per channel and combined in a fixed order
#pragma unroll
  for (int u = 0; u < WPT; ++u) {
    const int i = tid + u * nthr, j = i / WS, kc = i - j * WS, k = k0 + kc;
    if (i < TJ * WS) w_l[i] = (j < J && kc < TK && k < K) ? wreg[u] : 0.f;
  }
  if (PRO && tid < TJ * PS) {
    const int j = tid / PS, sub = psub;
    double t0 = 0.0, t1 = 0.0;
    if (j < J) {
      // block-tail partials [J][N][npart][3]: {sum g, sum g*xhat2, sum g*xhat_r} (PRO 2), or the
      // depthwise backward's IN partials [J][N][npart][2] (PRO 1); a lane's share (i = sub,
      // sub + PS, ..., up to 40 partials at 48^3) in batches of PB clamped unconditional loads
      // (the first batch requested above): one memory round trip per batch (same order of the adds)
      if constexpr (EP) {
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const bool ok = sub + u * PS < npart;
          t0 += ok ? pa0[u] : 0.0;
          t1 += ok ? pa1[u] : 0.0;
        }
      }
      for (int i0 = sub + (EP ? PB * PS : 0); i0 < npart; i0 += PB * PS) {
        double a0[PB], a1[PB];
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const int i = min(i0 + u * PS, npart - 1);
          a0[u] = pp[i * pst];
          a1[u] = pp[i * pst + po1];
        }
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const bool ok = i0 + u * PS < npart;
          t0 += ok ? a0[u] : 0.0;
          t1 += ok ? a1[u] : 0.0;
        }
      }
    }
    psum[tid * 2] = t0;
    psum[tid * 2 + 1] = t1;
  }
  __syncthreads();
  if (PRO && tid < TJ) {
    float* o = coef + tid * 8;
    if (tid < J) {
      double t0 = 0.0, t1 = 0.0;
      for (int i = 0; i < PS; ++i) { t0 += psum[(tid * PS + i) * 2]; t1 += psum[(tid * PS + i) * 2 + 1]; }
      o[0] = q1 * q5;              // f = rstd * gamma
      o[1] = (float)(t0 / S);      // M1
      o[2] = q0;                   // mu
      o[3] = q1;                   // rstd
      o[4] = (float)(t1 / S);      // M2
      o[5] = q7;                   // rank-1 scale of the operand (yns < 0)
    } else {
      o[0] = o[1] = o[2] = o[3] = o[4] = o[5] = 0.f;
    }
  }
  if (PRO) __syncthreads();

  // 3. dY (PRO: formed from dpre as l3u_in_bwd_apply does), copy into the wave's LDS tile
  if (PRO) {
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) {
      const int j = 4 * jr + lk;
      const float* c = coef + j * 8;
      const float f = c[0], M1 = c[1], mu = c[2], rs = c[3], M2 = c[4];
      const bool ok = j < J && sd < s_hi;
      if (yk) yv[jr] = mul_rn(yv[jr], c[5]);   // the materialised operand's value, bit for bit
      if (PRO == 2) {   // g = dout * lrelu'(out), then the tail InstanceNorm backward
#pragma unroll
        for (int q = 0; q < 4; ++q) g[jr][q] = g[jr][q] * lrelu_d(ov[jr][q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) g[jr][q] = ok ? f * (g[jr][q] - M1 - (yv[jr][q] - mu) * rs * M2) : 0.f;
    }
  }
  // the wave's dY tile: all TJ rows, or (TJ = 32) 16 rows at a time, written again for the second
  // half after the first half's weight-gradient reads (half the LDS: at 64^3 three -> four
  // workgroups per CU)
  constexpr int TR = NJ == 2 ? 16 : TJ;   // rows of the wave's LDS tile
  float* tile = dyt_lds + (size_t)wave * TR * DS;
#pragma unroll
  for (int jr = 0; jr < TR / 4; ++jr)
    *reinterpret_cast<f4*>(tile + dyt_at(4 * jr + lk, lr)) = g[jr];

  if constexpr (!XL) load_xv();

  // 4. data gradient, one 16-row tile of dX at a time, from the registers
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) {
    f4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) {
      const float a = w_l[(4 * jr + lk) * WS + 16 * kt + lr];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = mfma4(a, g[jr][q], acc[q]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 16 * kt + 4 * lk + r;
      if (k < K && sd < s_hi) {
        float* dst = dxn + (long long)k * S + sd;
        f4 v = f4{acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
        if (accumulate) v += ldv4(dst);
        stv4(dst, v);
      }
    }
  }

  // 5. weight gradient: dY rows back from the wave's LDS tile in the A layout
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  f4 gw[NJ][NK];
#pragma unroll
  for (int a = 0; a < NJ; ++a)
#pragma unroll
    for (int b = 0; b < NK; ++b) gw[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  auto wgrad = [&](auto A) {   // rows 16 a .. 16 a + 15 of the dY tile (16 a - TJ + TR in LDS)
    constexpr int a = decltype(A)::value;
    constexpr int ar = TR == TJ ? a : 0;
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f4 av = *reinterpret_cast<const f4*>(tile + dyt_at(16 * ar + lr, 4 * gg + lk));
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < NK; ++b) gw[a][b] = mfma4(av[q], xv[gg][b][q], gw[a][b]);
    }
  };
  if constexpr (TR == TJ) {
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      f4 av[NJ];
#pragma unroll
      for (int a = 0; a < NJ; ++a)
        av[a] = *reinterpret_cast<const f4*>(tile + dyt_at(16 * a + lr, 4 * gg + lk));
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int a = 0; a < NJ; ++a)
#pragma unroll
          for (int b = 0; b < NK; ++b) gw[a][b] = mfma4(av[a][q], xv[gg][b][q], gw[a][b]);
    }
  } else {
    wgrad(std::integral_constant<int, 0>{});
    // the second 16 rows into the same tile once this wave's reads of the first are done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int jr = 0; jr < 4; ++jr)
      *reinterpret_cast<f4*>(tile + dyt_at(4 * jr + lk, lr)) = g[4 + jr];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    wgrad(std::integral_constant<int, 1>{});
  }

  // 6. fixed-order cross-wave reduction (reuses the dY tiles), in wave order: every wave parks
  // its partial tile and wave 0 adds them; with the half tiles the waves add into one buffer in
  // turn (the same order and sums)
  float* red = dyt_lds;
  if constexpr (TR == TJ) {
    __syncthreads();
#pragma unroll
    for (int a = 0; a < NJ; ++a)
#pragma unroll
      for (int b = 0; b < NK; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((wave * NJ + a) * NK + b) * 256 + r * 64 + l] = gw[a][b][r];
    __syncthreads();
    if (wave == 0) {
      float* o = part + (long long)blockIdx.x * J * K;
#pragma unroll
      for (int a = 0; a < NJ; ++a)
#pragma unroll
        for (int b = 0; b < NK; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = red[(a * NK + b) * 256 + r * 64 + l];
            for (int wv = 1; wv < nwv; ++wv) v += red[((wv * NJ + a) * NK + b) * 256 + r * 64 + l];
            const int jj = 16 * a + 4 * lk + r, kk = k0 + 16 * b + lr;
            if (jj < J && kk < K) o[(long long)jj * K + kk] = v;
          }
    }
  } else {
    static_assert(NJ * NK * 256 <= 4 * 16 * DS, "the reduction buffer fits the tiles of 4 waves");
    for (int wv = 0; wv < nwv; ++wv) {
      __syncthreads();
      if (wave == wv) {
#pragma unroll
        for (int a = 0; a < NJ; ++a)
#pragma unroll
          for (int b = 0; b < NK; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = ((a * NK + b) * 4 + r) * 64 + l;
              red[i] = wv == 0 ? gw[a][b][r] : red[i] + gw[a][b][r];
            }
      }
    }
    __syncthreads();
    if (wave == 0) {
      float* o = part + (long long)blockIdx.x * J * K;
#pragma unroll
      for (int a = 0; a < NJ; ++a)
#pragma unroll
        for (int b = 0; b < NK; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int jj = 16 * a + 4 * lk + r, kk = k0 + 16 * b + lr;
            if (jj < J && kk < K) o[(long long)jj * K + kk] = red[((a * NK + b) * 4 + r) * 64 + l];
          }
    }
  }
}

// The pointwise backward with ONE input channel (K = 1: the first block's conv1.pointwise,
// unet3d.py:163-167 with in_channels = 1) and the InstanceNorm-backward prologue (PRO 1):
//   dY[j][s]  = f_j (dpre[j][s] - M1_j - (y[j][s] - mu_j) rs_j M2_j)     (l3u_in_bwd_apply)
//   dX[s]     = sum_j W[j] dY[j][s]                                     (j in order, fp32 fma)
//   part[j]   = sum_{s in chunk} dY[j][s] X[s]                           (fixed-order tree)
// On the VALU: at K = 1 the MFMA tile is 15/16 padding and the fused kernel moved 16 dY rows
// through LDS for one output column.  A thread owns 4 voxels, a workgroup the pw_bwd_fused
// chunk of SCH voxels (same partial layout part[chunk][J][1]); rows 16 at a time (J <= 32).  A
// rank-1 y (yns < 0) is one stored channel, row j = rec[j][7] * it (the materialised values).
template <typename T, bool YK>
__global__ __launch_bounds__(128) void pw_bwd_k1_kernel(
    const float* __restrict__ dy, long long dyns, const T* __restrict__ yin, long long yns,
    const float* __restrict__ rec, const double* __restrict__ in_part, int npart,
    const T* __restrict__ x, long long xns, const float* __restrict__ w, float* __restrict__ dx,
    long long dxns, int accumulate, float* __restrict__ part, int N, int J, int S, int SCH, int nsc) {
  L3U_STAMP_SCOPE(107);
  __shared__ float coef[32 * 8];
  __shared__ double psum[32 * 4 * 2];
  __shared__ float wred[2][32];
  const int tid = threadIdx.x, l = tid & 63, wave = tid >> 6, nwv = blockDim.x >> 6;
  const int sc = blockIdx.x % nsc, n = blockIdx.x / nsc;
  const int s = sc * SCH + 4 * tid;
  const bool ok = s < S && 4 * tid < SCH;
  const int sdc = ok ? s : S - 4;   // clamped address of the lanes past the chunk / volume
  constexpr bool yk = YK;   // rank-1 y (yns < 0): a template flag, the other form keeps 16 y rows
  const float* dyn = dy + (long long)n * dyns;
  const T* yn = yin + (long long)n * (yk ? -yns : yns);
  // (0) the small operands first (vector loads complete in order: requested behind the tile they
  // were two more dependent round trips, the partials with a wait behind every predicated load):
  // 4 lanes per row take the row's IN-backward partials (PB per lane, clamped unconditional
  // loads, added in index order; rows past 16 and partials past 4 * PB are loaded later), the
  // lanes j < J the row's record and weight
  constexpr int PB = 12;
  const int sub = tid & 3, pr0 = min(tid >> 2, J - 1);
  const double* pp0 = in_part + ((long long)pr0 * N + n) * npart * 2;
  double2 pv[PB];
#pragma unroll
  for (int u = 0; u < PB; ++u) pv[u] = *reinterpret_cast<const double2*>(pp0 + min(sub + 4 * u, npart - 1) * 2);
  const int jq = min(tid, J - 1);
  const float* qr = rec + ((long long)n * J + jq) * kRec;
  const float q0 = qr[0], q1 = qr[1], q5 = qr[5], q7 = qr[7], qw = w[jq];
  // (1) the first 16 rows' streamed loads, unconditional at clamped addresses
  f4 g[16], yv[yk ? 1 : 16];
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto load_rows = [&](int j0) {
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int jc = min(j0 + jj, J - 1);
      g[jj] = ldv4(dyn + (long long)jc * S + sdc);
      if constexpr (!yk) yv[jj] = ldv4(yn + (long long)jc * S + sdc);
    }
    if constexpr (yk) yv[0] = ldv4(yn + sdc);
  };
  load_rows(0);
  const f4 xv = ldv4(x + (long long)n * xns + sdc);
  // (2) the partial sums: 4 lanes per row, combined in lane order
  for (int jr = tid >> 2; jr < J; jr += blockDim.x >> 2) {
    double t0 = 0.0, t1 = 0.0;
    const double* pp = in_part + ((long long)jr * N + n) * npart * 2;
    int i0 = sub;
    if (jr == tid >> 2) {   // the first pass: the batch requested in (0)
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const bool in = sub + 4 * u < npart;
        t0 += in ? pv[u].x : 0.0;
        t1 += in ? pv[u].y : 0.0;
      }
      i0 = sub + 4 * PB;
    }
    for (; i0 < npart; i0 += 4 * PB) {
      double2 v[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) v[u] = *reinterpret_cast<const double2*>(pp + min(i0 + 4 * u, npart - 1) * 2);
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const bool in = i0 + 4 * u < npart;
        t0 += in ? v[u].x : 0.0;
        t1 += in ? v[u].y : 0.0;
      }
    }
    psum[(jr * 4 + sub) * 2] = t0;
    psum[(jr * 4 + sub) * 2 + 1] = t1;
  }
  __syncthreads();
  L3U_STAMP_MARK(0);
  if (tid < J) {   // J <= 32 < blockDim.x
    double t0 = 0.0, t1 = 0.0;
    for (int i = 0; i < 4; ++i) { t0 += psum[(tid * 4 + i) * 2]; t1 += psum[(tid * 4 + i) * 2 + 1]; }
    float* o = coef + tid * 8;
    o[0] = q1 * q5;              // f = rstd * gamma
    o[1] = (float)(t0 / S);      // M1
    o[2] = q0;                   // mu
    o[3] = q1;                   // rstd
    o[4] = (float)(t1 / S);      // M2
    o[5] = q7;                   // rank-1 scale
    o[6] = qw;                   // W[j][0]
  }
  __syncthreads();
  f4 dxa = z4;
  float pw[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) pw[j] = 0.f;
  const f4 y1 = yv[0];
  // rows 16 H .. 16 H + 15 (compile-time indices: registers); rows j >= J contribute zeros (a
  // select, no branch: the rows' arithmetic and the reductions below interleave)
  auto rows = [&](auto H) {
    constexpr int h = decltype(H)::value;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int j = 16 * h + jj;
      const bool rok = ok && j < J;
      const float* c = coef + min(j, J - 1) * 8;
      const float f = c[0], M1 = c[1], mu = c[2], rs = c[3], M2 = c[4];
      f4 yj;
      if constexpr (yk) yj = mul_rn(y1, c[5]); else yj = yv[jj];
      f4 d;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = rok ? f * (g[jj][q] - M1 - (yj[q] - mu) * rs * M2) : 0.f;
      const float wj = c[6];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dxa[q] = fmaf(wj, d[q], dxa[q]);
        pw[j] = fmaf(d[q], xv[q], pw[j]);
      }
    }
  };
  L3U_STAMP_MARK(1);
  rows(std::integral_constant<int, 0>{});
  if (J > 16) {   // uniform
    load_rows(16);
    rows(std::integral_constant<int, 1>{});
  }
  if (ok) {
    float* dst = dx + (long long)n * dxns + s;
    if (accumulate) dxa += ldv4(dst);
    *reinterpret_cast<f4*>(dst) = dxa;
  }
  // weight-gradient partial of the chunk: xor tree over the wave, then the waves in order (the 16
  // rows of a half reduced together: their shuffle chains interleave)
  auto reduce_half = [&](auto H) {
    constexpr int h = decltype(H)::value;
    float v[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = pw[16 * h + jj];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) v[jj] += __shfl_xor(v[jj], o, 64);
    if (l == 0) {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj)
        if (16 * h + jj < J) wred[wave][16 * h + jj] = v[jj];
    }
  };
  reduce_half(std::integral_constant<int, 0>{});
  if (J > 16) reduce_half(std::integral_constant<int, 1>{});
  __syncthreads();
  for (int j = tid; j < J; j += blockDim.x) {
    float v = wred[0][j];
    for (int k = 1; k < nwv; ++k) v += wred[k][j];
    part[(long long)blockIdx.x * J + j] = v;
  }
}

// Fused 1x1-conv backward for wide J (J = 16 * JT * NWV: 64 / 128 for the 12^3 / 6^3 levels,
// and the ConvTranspose3d(k2, s2) backward, J = Co*8 up to 512), latency-bound shapes: one
// workgroup of NWV waves per (64-voxel tile, 16 columns of K).  Wave w owns the dY rows
// [w*16*JT, +16*JT): it forms its share of the data gradient (split-J partial, combined across the
// waves through LDS in wave order) and the weight-gradient rows of the same dY rows over the
// tile.  dY is read in both MFMA layouts straight from global (the second read hits L1/L2; each
// wave needs only its own rows); PRO 1 applies the InstanceNorm backward to both.
// GATHER 1/2 (ConvTranspose3d): dY row j = co*8 + abc is read in place from the up-sampled
// gradient (load_x4 GATHER; 2 = scalar gathers for W % 4 != 0); the weights are stored W[k][j]
// (the ConvTranspose3d weight [Ci][Co*8]) and so are the partials; bpart != NULL receives the
// bias partials sum_{tile, abc} dY[co] per (tile, co) from the K-tile-0 workgroups.
// Partials are per 64-voxel tile: part[N * ceil(S/64)][J][K] ([K][J] for GATHER).
// the second problem of a paired wide launch (l3u_pw_bwd2): same J, N, S; its own dY, X, W, dX,
// K, accumulate flag and partials (blockIdx.z == 1)
template <typename T>
struct WideSecond {
  const float* dy; long long dyns; const T* x; long long xns; const float* w; float* dx;
  long long dxns; int accumulate; float* part; int K;
};

template <typename T, int JT, int NWV, int PRO, int GATHER, bool MT = false>
__global__ __launch_bounds__(64 * NWV) void pw_bwd_wide_kernel(
    const float* __restrict__ dy, long long dyns, const T* __restrict__ yin, long long yns,
    const float* __restrict__ rec, const double* __restrict__ in_part, int npart,
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    float* __restrict__ dx, long long dxns, int accumulate, float* __restrict__ part,
    float* __restrict__ bpart, int N, int J, int K, int S, int Hq, int Wq, int tpb,
    WideSecond<T> p2 = WideSecond<T>{}) {
  L3U_STAMP_SCOPE(105);
  if (blockIdx.z == 1) {   // paired launch, second problem (PRO 0, no gather)
    dy = p2.dy; dyns = p2.dyns; x = p2.x; xns = p2.xns; w = p2.w; dx = p2.dx; dxns = p2.dxns;
    accumulate = p2.accumulate; part = p2.part; K = p2.K;
  }
  if ((int)blockIdx.y * 16 >= K) return;   // the narrower problem's unused column blocks
  constexpr int JW = 16 * JT;                 // dY rows per wave
  constexpr bool GV = GATHER != 2;            // vector loads
  constexpr bool G = GATHER != 0;
  __shared__ __attribute__((aligned(16))) float coef[PRO ? 128 * 8 : 1];
  __shared__ __attribute__((aligned(16))) float red[NWV][16 * 64];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  // workgroup = tpb consecutive 64-voxel tiles of one sample (weight-gradient partials summed
  // over them in registers: one partial per workgroup)
  // MT = false: one tile per workgroup (tpb == 1, compile-time: the latency-bound levels keep
  // the single-tile schedule and registers)
  if (!MT) tpb = 1;
  const int ntile = (S + 63) / 64, nblk = (ntile + tpb - 1) / tpb;
  const int tb = blockIdx.x % nblk, n = blockIdx.x / nblk, k0 = blockIdx.y * 16;
  const int t0 = tb * tpb, t1 = min(ntile, t0 + tpb), jb = wave * JW;
  const float* dyn = dy + (long long)n * dyns;
  const T* xn = x + (long long)n * xns;

  f4 gw[JT];
  float bsum[JT];
#pragma unroll
  for (int t = 0; t < JT; ++t) { gw[t] = f4{0.f, 0.f, 0.f, 0.f}; bsum[t] = 0.f; }
  float wa[JT * 4];   // the weights W[jb + 4jr + lk][k0 + lr]
#pragma unroll
  for (int jr = 0; jr < JT * 4; ++jr) {
    const int j = jb + 4 * jr + lk, k = k0 + lr;
    wa[jr] = k < K ? (G ? w[(long long)k * J + j] : w[(long long)j * K + k]) : 0.f;
  }
  // PRO: the InstanceNorm-backward partials (the first NPB of them) and the records are small
  // operands as well, requested before the streamed tile: loads complete in order, so requested
  // behind it they were a second dependent round trip (plus one per seq_sum batch, whose
  // predicated loads each waited for everything in flight)
  constexpr int NPB = JT == 1 ? 8 : 4;   // the 12^3 IN-fused depthwise backward leaves 6 per (n, c)
  const int pc = min(tid, J - 1);
  const double* pp = PRO ? in_part + ((long long)pc * N + n) * npart * 2 : nullptr;
  double pa[PRO ? NPB : 1][2];
  float q0 = 0.f, q1 = 0.f, q5 = 0.f;
  if constexpr (PRO != 0) {
#pragma unroll
    for (int u = 0; u < NPB; ++u) {
      const int i = min(u, npart - 1);
      pa[u][0] = pp[i * 2];
      pa[u][1] = pp[i * 2 + 1];
    }
    const float* q = rec + ((long long)n * J + pc) * kRec;
    q0 = q[0]; q1 = q[1]; q5 = q[5];
  }

  for (int tile = t0; tile < t1; ++tile) {
    const int v0 = tile * 64;
    // streamed loads first: dY in the data-gradient B layout (rows jb + 4jr + lk, voxels
    // v0 + 4lr..), dY in the weight-gradient A layout (rows jb + 16t + lr, voxels v0 + 16g + 4lk..),
    // X in the B layout (rows k0 + lr)
    f4 gd[JT * 4], ga[JT][4], yd[PRO ? JT * 4 : 1], ya[PRO ? JT : 1][4], xb[4];
    const int vd = v0 + 4 * lr;
    // accumulate: the dX values this lane adds to in the epilogue (waves 0..3: k0 + 4lk + wave),
    // requested first (requested in the epilogue they were one more dependent round trip)
    f4 dprev = {0.f, 0.f, 0.f, 0.f};
    if (GV && accumulate)
      dprev = ldv4(dx + (long long)n * dxns + (long long)min(k0 + 4 * lk + (wave & 3), K - 1) * S + min(vd, S - 4));
#pragma unroll
    for (int jr = 0; jr < JT * 4; ++jr) gd[jr] = load_x4<GV, G>(dyn, jb + 4 * jr + lk, J, vd, S, S, Hq, Wq);
#pragma unroll
    for (int t = 0; t < JT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        ga[t][g] = load_x4<GV, G>(dyn, jb + 16 * t + lr, J, v0 + 16 * g + 4 * lk, S, S, Hq, Wq);
    if (PRO) {
      const T* yn = yin + (long long)n * yns;
#pragma unroll
      for (int jr = 0; jr < JT * 4; ++jr) yd[jr] = load_x4<true, false>(yn, jb + 4 * jr + lk, J, vd, S, S, 0, 0);
#pragma unroll
      for (int t = 0; t < JT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          ya[t][g] = load_x4<true, false>(yn, jb + 16 * t + lr, J, v0 + 16 * g + 4 * lk, S, S, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
      xb[g] = load_x4<GV, false>(xn, k0 + lr, K, v0 + 16 * g + 4 * lk, S, S, 0, 0);

    if (PRO && tile == t0) {
      // per-row InstanceNorm-backward coefficients (rows < J <= 128); the partials summed in
      // index order (seq_sum's order: same bits), the ones past NPB (none at 12^3 / 6^3: a loop
      // of dependent loads otherwise) loaded here
      if (tid < J) {
        double t[2] = {0.0, 0.0};
#pragma unroll
        for (int u = 0; u < NPB; ++u)
          if (u < npart) { t[0] += pa[u][0]; t[1] += pa[u][1]; }
        for (int i = NPB; i < npart; ++i) { t[0] += pp[i * 2]; t[1] += pp[i * 2 + 1]; }
        float* o = coef + tid * 8;
        o[0] = q1 * q5;
        o[1] = (float)(t[0] / S);
        o[2] = q0;
        o[3] = q1;
        o[4] = (float)(t[1] / S);
      }
      __syncthreads();
    }
    if (PRO) {
#pragma unroll
      for (int jr = 0; jr < JT * 4; ++jr) {
        const float* c = coef + (jb + 4 * jr + lk) * 8;
        const float f = c[0], M1 = c[1], mu = c[2], rs = c[3], M2 = c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          gd[jr][q] = vd + q < S ? f * (gd[jr][q] - M1 - (yd[jr][q] - mu) * rs * M2) : 0.f;
      }
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        const float* c = coef + (jb + 16 * t + lr) * 8;
        const float f = c[0], M1 = c[1], mu = c[2], rs = c[3], M2 = c[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int v = v0 + 16 * g + 4 * lk;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            ga[t][g][q] = v + q < S ? f * (ga[t][g][q] - M1 - (ya[t][g][q] - mu) * rs * M2) : 0.f;
        }
      }
    }

    // data gradient: this wave's split-J partial of dX[k0 + 4lk + r][vd + q]
    f4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jr = 0; jr < JT * 4; ++jr)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = mfma4(wa[jr], gd[jr][q], acc[q]);
    // weight gradient of the wave's rows over the tile, accumulated over the workgroup's tiles
#pragma unroll
    for (int t = 0; t < JT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) gw[t] = mfma4(ga[t][g][q], xb[g][q], gw[t]);
    if (G && bpart != nullptr && blockIdx.y == 0) {
      // bias partial of co = j / 8: row sums over the tile (lanes lk), then the 8 rows abc of
      // each co (lanes lr & 7), both in a fixed xor-tree order; tiles added in order
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        float sum = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) sum += (ga[t][g][0] + ga[t][g][1]) + (ga[t][g][2] + ga[t][g][3]);
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        sum += __shfl_xor(sum, 1, 64);
        sum += __shfl_xor(sum, 2, 64);
        sum += __shfl_xor(sum, 4, 64);
        bsum[t] += sum;
      }
    }
    // combine the NWV split-J partials in wave order; waves 0..3 then store rows r == wave
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][(q * 4 + r) * 64 + l] = acc[q][r];
    __syncthreads();
    L3U_STAMP_MARK(1);
    if (wave < 4) {
      const int r = wave;
      const int k = k0 + 4 * lk + r;
      f4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = (q * 4 + r) * 64 + l;
        float sum = red[0][i];
#pragma unroll
        for (int wv = 1; wv < NWV; ++wv) sum += red[wv][i];
        v[q] = sum;
      }
      if (k < K) {
        float* dst = dx + (long long)n * dxns + (long long)k * S + vd;
        if (GV) {
          if (vd < S) {
            if (accumulate) v += dprev;
            stv4(dst, v);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (vd + q < S) st1(dst + q, accumulate ? ld1(dst + q) + v[q] : v[q]);
        }
      }
    }
    if (tile + 1 < t1) __syncthreads();   // red is rewritten by the next tile
  }
  float* o = part + (long long)blockIdx.x * J * K;
#pragma unroll
  for (int t = 0; t < JT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jb + 16 * t + 4 * lk + r, k = k0 + lr;
      if (k < K) o[G ? (long long)k * J + j : (long long)j * K + k] = gw[t][r];
    }
  if (G && bpart != nullptr && blockIdx.y == 0) {
#pragma unroll
    for (int t = 0; t < JT; ++t)
      if (lk == 0 && (lr & 7) == 0) bpart[(long long)blockIdx.x * (J / 8) + (jb + 16 * t + lr) / 8] = bsum[t];
  }
}

// ConvTranspose3d(k2, s2) data gradient in the x-PAIR layout (even W):
//   dX[ci][z,y,x] = sum_{co,a,b,c} w[ci][co*8 + 4a+2b+c] dY[co][2z+a][2y+b][2x+c]
// MFMA column j = input voxel PAIR q (x = 2xp, 2xp+1): for one (co, a, b) the four dY values of
// the pair, (2x, c0) (2x, c1) (2x+1, c0) (2x+1, c1), are ONE contiguous float4 of an up-sampled row,
// so lane (lr, lk) loads dY[co0 + lk][2z+a][2y+b][4xp .. 4xp+3] of pair q0 + lr (16 lanes: 256 B of
// one row run, no gather, no redundant bytes) and feeds it to four MFMAs: elements 0/1 (c = 0/1)
// into the even-voxel accumulator, 2/3 into the odd one, with the weights w[ci][co*8+4a+2b+c] as
// the A operand.  KW waves split the co range (interleaved co quads) and combine through LDS in
// wave order (deterministic).  Replaces the gathered-GEMM form for the model's decoder shapes.
template <int NC, int KW>
L3U_DEV void convt_dx_pair_body(int bx, int by, int bz,
    const float* __restrict__ dy, long long dyns, const float* __restrict__ w, float* __restrict__ dx,
    long long dxns, int Ci, int Co, int D, int H, int W) {
  __shared__ __attribute__((aligned(16))) float red[KW][NC * 2 * 4][64];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int WP = W >> 1, P = D * H * WP;
  const long long S = (long long)D * H * W, S8 = 8 * S;
  const int q = bx * 16 + lr, ci0 = by * 16 * NC, n = bz;
  const bool ok = q < P;
  const int qq = ok ? q : 0;
  const int xp = qq % WP, t = qq / WP, y = t % H, z = t / H;
  const float* dyn = dy + (long long)n * dyns;
  // row offsets of the four (a, b) up-sampled rows of this pair (within one co plane)
  long long ro[4];
#pragma unroll
  for (int ab = 0; ab < 4; ++ab)
    ro[ab] = ((long long)(2 * z + (ab >> 1)) * (2 * H) + (2 * y + (ab & 1))) * (2 * W) + 4 * xp;
  f4 ae[NC], ao[NC];
#pragma unroll
  for (int m = 0; m < NC; ++m) ae[m] = ao[m] = f4{0.f, 0.f, 0.f, 0.f};
  const int nq = (Co + 3) >> 2;
  // UB co quads of the wave per batch with every load of the batch in flight before the first
  // MFMA (one memory round trip per batch, not per co quad): clamped unconditional addresses, the
  // out-of-range operands zeroed after the load (a predicated load makes hipcc branch around it and
  // wait for everything in flight); the MFMAs in the same order as one quad at a time
  constexpr int UB = 4;
  for (int cq0 = wave; cq0 < nq; cq0 += UB * KW) {
    f4 v[UB][4];
    float wv[UB][NC][8];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int co = min(4 * (cq0 + u * KW) + lk, Co - 1);
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) v[u][ab] = *reinterpret_cast<const f4*>(dyn + (long long)co * S8 + ro[ab]);
#pragma unroll
      for (int m = 0; m < NC; ++m) {
        const int ci = min(ci0 + 16 * m + lr, Ci - 1);
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[u][m][e] = w[(long long)ci * Co * 8 + co * 8 + e];
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int co = 4 * (cq0 + u * KW) + lk;
      const bool cok = co < Co;
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) v[u][ab] = (ok && cok) ? v[u][ab] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < NC; ++m) {
        const bool wok = cok && ci0 + 16 * m + lr < Ci;
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[u][m][e] = wok ? wv[u][m][e] : 0.f;
      }
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int m = 0; m < NC; ++m) {
          ae[m] = mfma4(wv[u][m][2 * ab], v[u][ab][0], ae[m]);
          ae[m] = mfma4(wv[u][m][2 * ab + 1], v[u][ab][1], ae[m]);
          ao[m] = mfma4(wv[u][m][2 * ab], v[u][ab][2], ao[m]);
          ao[m] = mfma4(wv[u][m][2 * ab + 1], v[u][ab][3], ao[m]);
        }
    }
  }
  if (KW > 1) {
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wave][(m * 2) * 4 + r][l] = ae[m][r];
        red[wave][(m * 2 + 1) * 4 + r][l] = ao[m][r];
      }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float se = red[0][(m * 2) * 4 + r][l], so = red[0][(m * 2 + 1) * 4 + r][l];
#pragma unroll
        for (int wv2 = 1; wv2 < KW; ++wv2) {
          se += red[wv2][(m * 2) * 4 + r][l];
          so += red[wv2][(m * 2 + 1) * 4 + r][l];
        }
        ae[m][r] = se;
        ao[m][r] = so;
      }
  }
  if (!ok) return;
  float* dxn = dx + (long long)n * dxns + ((long long)z * H + y) * W + 2 * xp;
#pragma unroll
  for (int m = 0; m < NC; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ci = ci0 + 16 * m + 4 * lk + r;
      if (ci < Ci) *reinterpret_cast<f2_t*>(dxn + (long long)ci * S) = f2_t{ae[m][r], ao[m][r]};
    }
}

template <int NC, int KW>
__global__ __launch_bounds__(64 * KW) void convt_dx_pair_kernel(
    const float* __restrict__ dy, long long dyns, const float* __restrict__ w, float* __restrict__ dx,
    long long dxns, int Ci, int Co, int D, int H, int W) {
  L3U_STAMP_SCOPE(106);
  convt_dx_pair_body<NC, KW>(blockIdx.x, blockIdx.y, blockIdx.z, dy, dyns, w, dx, dxns, Ci, Co, D, H, W);
}

// ConvTranspose3d(k2, s2) weight and bias gradients in the same x-pair layout (even W):
//   part[chunk][ci][co*8 + 4a+2b+c] = sum_{s in chunk} x[ci][s] dY[co][2z+a][2y+b][2x+c]
// The MFMA k-dimension is the voxel.  Lane (lr, lk) loads the float4 of up-sampled row
// (co = 4g + lr/4, a, b = lr%4) at voxel pair lk of the step (both voxels of the pair, c = 0 / 1):
// component (even, c) is B[k = lk][column lr] of the c-MFMA on the pair's even voxel, (odd, c) of
// the one on its odd voxel, with A = x[ci][that voxel] (a float2 per lane).  Columns c = 0 and
// c = 1 accumulate separately: acc[m][g][c] holds part[ci0+16m+4lk+r][(4g+lr/4)*8 + 2*(lr%4)+c].
// Bias partial bsum[chunk][co] = sum of every dY value of co over the chunk's up-sampled voxels.
// Same partial layout and chunking as pw_bwd_weight_kernel's GATHER form.
template <typename T, int NJ, int NG>
L3U_DEV void convt_dw_pair_body(int bx, int by,
    const T* __restrict__ x, long long xns, const float* __restrict__ dy, long long dyns,
    float* __restrict__ part, float* __restrict__ bsum, int Ci, int Co, int D, int H, int W,
    int SCH, int nsc) {
  __shared__ __attribute__((aligned(16))) float red[4][NJ * NG * 2 * 4][64];
  __shared__ float bred[4][NG * 4];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int WP = W >> 1;
  const long long S = (long long)D * H * W, S8 = 8 * S;
  const int sc = bx % nsc, n = bx / nsc;
  const int ngb = (Co + 4 * NG - 1) / (4 * NG);
  const int ci0 = (by / ngb) * 16 * NJ, g0 = (by % ngb) * NG;
  const int p_lo = sc * (SCH / 2), p_hi = min((int)(S / 2), p_lo + SCH / 2);
  const int ab = lr & 3, a_ = ab >> 1, b_ = ab & 1;
  const float* dyn = dy + (long long)n * dyns;
  const T* xn = x + (long long)n * xns;
  f4 acc[NJ][NG][2];
#pragma unroll
  for (int m = 0; m < NJ; ++m)
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[m][g][0] = acc[m][g][1] = f4{0.f, 0.f, 0.f, 0.f};
  float bacc[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) bacc[g] = 0.f;
  // UB voxel-pair steps per batch, every load of the batch in flight before the first MFMA (as in
  // convt_dx_pair_body); steps past the chunk load clamped addresses and add zeros
  constexpr int UB = NJ * NG <= 2 ? 8 : 4;
  for (int pb0 = p_lo + 4 * wave; pb0 < p_hi; pb0 += UB * 16) {
    f4 v[UB][NG];
    f2_t xv[UB][NJ];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int p = pb0 + 16 * u + lk;
      const int pc = p < p_hi ? p : p_lo;
      const int xp = pc % WP, t = pc / WP, y = t % H, z = t / H;
      const long long ro = ((long long)(2 * z + a_) * (2 * H) + (2 * y + b_)) * (2 * W) + 4 * xp;
      const long long xo = ((long long)z * H + y) * W + 2 * xp;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int co = min(4 * (g0 + g) + (lr >> 2), Co - 1);
        v[u][g] = *reinterpret_cast<const f4*>(dyn + (long long)co * S8 + ro);
      }
#pragma unroll
      for (int m = 0; m < NJ; ++m) xv[u][m] = ldv2(xn + (long long)min(ci0 + 16 * m + lr, Ci - 1) * S + xo);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const bool ok = pb0 + 16 * u + lk < p_hi;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const bool vok = ok && 4 * (g0 + g) + (lr >> 2) < Co;
        const f4 vg = vok ? v[u][g] : f4{0.f, 0.f, 0.f, 0.f};
        bacc[g] += (vg[0] + vg[1]) + (vg[2] + vg[3]);
#pragma unroll
        for (int m = 0; m < NJ; ++m) {
          const f2_t xm = (ok && ci0 + 16 * m + lr < Ci) ? xv[u][m] : f2_t{0.f, 0.f};
          acc[m][g][0] = mfma4(xm[0], vg[0], acc[m][g][0]);
          acc[m][g][1] = mfma4(xm[0], vg[1], acc[m][g][1]);
          acc[m][g][0] = mfma4(xm[1], vg[2], acc[m][g][0]);
          acc[m][g][1] = mfma4(xm[1], vg[3], acc[m][g][1]);
        }
      }
    }
  }
  // fixed-order cross-wave reduction
#pragma unroll
  for (int m = 0; m < NJ; ++m)
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][((m * NG + g) * 2 + c) * 4 + r][l] = acc[m][g][c][r];
  if (bsum != nullptr && ci0 == 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {   // lanes of one co: lr%4 (a, b) and lk, in a fixed xor order
      float bv = bacc[g];
      bv += __shfl_xor(bv, 1, 64);
      bv += __shfl_xor(bv, 2, 64);
      bv += __shfl_xor(bv, 16, 64);
      bv += __shfl_xor(bv, 32, 64);
      if (lk == 0 && ab == 0) bred[wave][g * 4 + (lr >> 2)] = bv;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const int K = Co * 8;
    float* o = part + (long long)bx * Ci * K;
#pragma unroll
    for (int m = 0; m < NJ; ++m)
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = ((m * NG + g) * 2 + c) * 4 + r;
            const float vsum = ((red[0][i][l] + red[1][i][l]) + red[2][i][l]) + red[3][i][l];
            const int ci = ci0 + 16 * m + 4 * lk + r, co = 4 * (g0 + g) + (lr >> 2);
            if (ci < Ci && co < Co) o[(long long)ci * K + co * 8 + 2 * ab + c] = vsum;
          }
    if (bsum != nullptr && ci0 == 0 && l < NG * 4) {
      const int co = 4 * g0 + l;
      if (co < Co)
        bsum[(long long)bx * Co + co] = ((bred[0][l] + bred[1][l]) + bred[2][l]) + bred[3][l];
    }
  }
}

template <typename T, int NJ, int NG>
__global__ __launch_bounds__(256) void convt_dw_pair_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ dy, long long dyns,
    float* __restrict__ part, float* __restrict__ bsum, int Ci, int Co, int D, int H, int W,
    int SCH, int nsc) {
  L3U_STAMP_SCOPE(109);
  convt_dw_pair_body<T, NJ, NG>(blockIdx.x, blockIdx.y, x, xns, dy, dyns, part, bsum, Ci, Co, D, H, W,
                                SCH, nsc);
}

// Both pair-layout ConvTranspose3d backward halves in ONE launch (the 6^3 decoder input, where
// each is a ~10 us latency-bound launch): workgroups [0, nA) take the data gradient (grid gx x
// gy x gz of convt_dx_pair_kernel<NC, 4>), the rest the weight / bias partials (grid gwx x gwy
// of convt_dw_pair_kernel).  The two read the same dY and are independent; per-workgroup work and
// results are those of the two launches, bit for bit.
template <typename T, int NC, int NJ, int NG>
__global__ __launch_bounds__(256) void convt_pair_bwd_kernel(
    const float* __restrict__ dy, long long dyns, const float* __restrict__ w, float* __restrict__ dx,
    long long dxns, const T* __restrict__ x, long long xns, float* __restrict__ part,
    float* __restrict__ bsum, int Ci, int Co, int D, int H, int W, int SCH, int nsc, int gx, int gy,
    int nA, int gwx) {
  L3U_STAMP_SCOPE(108);
  const int b = blockIdx.x;
  if (b < nA) {
    convt_dx_pair_body<NC, 4>(b % gx, (b / gx) % gy, b / (gx * gy), dy, dyns, w, dx, dxns, Ci, Co, D, H, W);
  } else {
    const int k = b - nA;
    convt_dw_pair_body<T, NJ, NG>(k % gwx, k / gwx, x, xns, dy, dyns, part, bsum, Ci, Co, D, H, W, SCH, nsc);
  }
}

constexpr int kPwSchMax = 256;   // 4-wave sweeps at >= 64K voxels: config 5 -115 us (the 64^3 J = 32 tails hold 85 KB of LDS as 8-wave sweeps: one workgroup per CU), 48^3 -3 us
constexpr int kPwNswMax = 1;
constexpr int kPwSchMid = 256;   // voxel chunk of the mid-size levels (4096 <= S < 65536: 24^3); 512: +10 us/step
constexpr int pw_sch(int S) {
  return S >= 65536 ? kPwSchMax : (S >= 4096 ? kPwSchMid : (S >= 1024 ? 512 : 256));
}
// The chunk invariant.  A chunk is ONE workgroup sweep of every kernel that writes chunk partials
// (part[N * nsc][J][K], nsc = ceil(S / SCH)): pw_bwd_fused_kernel runs SCH / 64 waves (1..8),
// pw_bwd_k1_kernel SCH / 4 threads, which must be whole waves (its xor-tree reduction reads all 64
// lanes) and at most its 128-thread launch bound (pw_bwd_weight_kernel and the ConvTranspose3d
// weight kernels bound their loops by the chunk and take any size).  A chunk size breaking this
// left lanes of the K = 1 kernel's reduction unwritten (round 5: 192-voxel chunks, 48-thread
// workgroups, gave NaN weight gradients at the 64^3 first block).  Every chunk size pw_sch can
// return is checked here, l3u_pw_bwd_chunk reports it to the host (tests/test_capi.py), and the
// launches re-check their own form.
constexpr bool pw_chunk_ok(int SCH) {
  return SCH % 256 == 0 && SCH / 64 >= 1 && SCH / 64 <= 8 && SCH / 4 <= 128;
}
static_assert(pw_chunk_ok(pw_sch(1)) && pw_chunk_ok(pw_sch(1024)) && pw_chunk_ok(pw_sch(4096)) &&
              pw_chunk_ok(pw_sch(65536)), "every pointwise-backward chunk size keeps the invariant");

// voxel sub-tiles per wave of pw_fwd_kernel: fewer for narrow outputs so that big volumes
// still launch enough workgroups (>= 4 per CU at one sample)
int pw_nsw(int NC) { const int n = 4 / NC; return n < kPwNswMax ? n : kPwNswMax; }

constexpr int kPwMinBlocks = 1024;   // measured: 0 / 512 / 1024 within 2 us, 1024 best
constexpr int kPwKsMinK = 0;
constexpr int kConvtKsMinK = 64;   // ConvTranspose3d forward: shallower K takes the unsplit kernel (up3: 19.3 -> 14.5 us)
constexpr int kPwks8MaxWg = 1024;   // grids up to this many workgroups take all k-steps in flight
// K split across the 4 waves (pw_fwd_ks_kernel) for small volumes with a deep enough reduction
constexpr int kPwKsMaxS = 32768;
bool pw_use_ks(int S, int K) { return S < kPwKsMaxS && K >= kPwKsMinK; }
// the one-wave form (pw_fwd_w1_kernel) of the K-split range from this volume on
#ifndef L3U_PW_W1
#define L3U_PW_W1 1
#endif
constexpr bool kPwW1 = L3U_PW_W1 != 0;
constexpr int kPwW1MinS = 4096;
constexpr int kPwW1MaxK = 32;   // K = 64 (the 24^3 decoder pair 64 -> 32): 16.2 -> 18.0 us, kept on pw_fwd_ks

}  // namespace

namespace {

template <typename T>
struct PwSecond {   // the second problem of a paired launch: same K, Nout, S, N and options
  const T* x; long long xns; const float* w; T* y; long long yns; float* stat;
};

template <typename T>
int pw_launch(const T* x, long long x_nstride, const float* w, int w_layout, const float* bias,
              T* y, long long y_nstride, int accumulate, float* stat_part, int N, int K,
              int Nout, int S, int xm, int Dq, int Hq, int Wq, hipStream_t stream,
              const PwSecond<T>* sec = nullptr) {
  const PwSecond<T> z2{nullptr, 0, nullptr, nullptr, 0, nullptr};
  const PwSecond<T>& p2 = sec ? *sec : z2;
  const int NZ = sec ? 2 * N : N;
  // xm: 0 plain GEMM, 1 ConvTranspose3d scatter epilogue, 2 X gathered from the up-sampled
  // ConvTranspose3d gradient; (Dq, Hq, Wq) = the low-resolution volume for xm != 0
  L3U_REQUIRE(N > 0 && K > 0 && Nout > 0 && S > 0);
  const bool vec = (S % 4 == 0) && (x_nstride % 4 == 0) && (y_nstride % 4 == 0) &&
                   (xm == 0 || Wq % 4 == 0);
  if (kPwW1 && pw_use_ks(S, K) && xm == 0 && vec && S >= kPwW1MinS && K <= kPwW1MaxK) {
    // one-wave tiles with the whole reduction in registers (pw_fwd_w1_kernel)
    const int nsb = (S + 63) / 64;
    const int NC = Nout <= 16 ? 1 : 2;
    dim3 grid(nsb, (Nout + 16 * NC - 1) / (16 * NC), NZ), block(64);
    const int KSn = K <= 16 ? 4 : 8;
#define PW1(NC_, KS_) hipLaunchKernelGGL((pw_fwd_w1_kernel<T, NC_, KS_>), grid, block, 0, stream, x, \
      x_nstride, w, w_layout, bias, y, y_nstride, accumulate, stat_part, K, Nout, S, nsb, p2.x, p2.xns, \
      p2.w, p2.y, p2.yns, p2.stat, N)
#define PW1_K(NC_) do { if (KSn == 4) PW1(NC_, 4); else PW1(NC_, 8); } while (0)
    if (NC == 1) PW1_K(1); else PW1_K(2);
#undef PW1_K
#undef PW1
    L3U_CHECK_LAUNCH();
  }
  if (pw_use_ks(S, K) && !(xm == 1 && K < kConvtKsMinK)) {
    // co tile: as wide as possible while keeping >= 256 workgroups
    const int nsb = (S + 63) / 64;
    int NC = Nout <= 16 ? 1 : (Nout <= 32 ? 2 : 4);
    while (NC > 1 && (long long)nsb * ((Nout + 16 * NC - 1) / (16 * NC)) * N < 256) NC >>= 1;
    const size_t lds = 4 * 64 * (size_t)NC * 16 * sizeof(float);
    dim3 grid(nsb, (Nout + 16 * NC - 1) / (16 * NC), NZ), block(256);
    // the whole grid in one round of waves: the latency-bound form (all k-steps of a wave in flight)
    const bool ks8 = NC <= 2 && xm != 2 && (long long)grid.x * grid.y * grid.z <= kPwks8MaxWg;
#define PWK(NC_, V_, X_) do { if (ks8) hipLaunchKernelGGL((pw_fwd_ks_kernel<T, NC_, V_, X_, 8>), grid, block, lds, \
      stream, x, x_nstride, w, w_layout, bias, y, y_nstride, accumulate, stat_part, K, Nout, S, nsb, Dq, Hq, Wq, \
      p2.x, p2.xns, p2.w, p2.y, p2.yns, p2.stat, N); \
      else hipLaunchKernelGGL((pw_fwd_ks_kernel<T, NC_, V_, X_, 4>), grid, block, lds, stream, \
      x, x_nstride, w, w_layout, bias, y, y_nstride, accumulate, stat_part, K, Nout, S, nsb, Dq, Hq, Wq, \
      p2.x, p2.xns, p2.w, p2.y, p2.yns, p2.stat, N); } while (0)
#define PWK_X(NC_, V_) do { if (xm == 1) PWK(NC_, V_, 1); else if (xm == 2) PWK(NC_, V_, 2); else PWK(NC_, V_, 0); } while (0)
#define PWK_V(NC_) do { if (vec) PWK_X(NC_, true); else PWK_X(NC_, false); } while (0)
    if (NC == 1) PWK_V(1);
    else if (NC == 2) PWK_V(2);
    else PWK_V(4);
#undef PWK_V
#undef PWK_X
#undef PWK
    L3U_CHECK_LAUNCH();
  }
  int CO_BLK = Nout <= 16 ? 16 : (Nout <= 32 ? 32 : 64);
  // narrower output tiles while the grid is short of kPwMinBlocks workgroups (the 24^3 ->
  // 48^3 ConvTranspose3d: 432 -> 864)
  while (CO_BLK > 16 && (long long)((S + 255) / 256) * ((Nout + CO_BLK - 1) / CO_BLK) * NZ <
                        kPwMinBlocks) CO_BLK >>= 1;
  const int NC = CO_BLK / 16, NSW = pw_nsw(NC), TSB = 256 * NSW;
  const int nsb = (S + TSB - 1) / TSB;
  const int WS = (CO_BLK % 32 == 16) ? CO_BLK : CO_BLK + 16;
  const int Kp = (K + 3) & ~3;
  size_t lds = (size_t)(Kp < 128 ? Kp : 128) * WS * sizeof(float);
  if (lds < 4 * CO_BLK * sizeof(float)) lds = 4 * CO_BLK * sizeof(float);
  L3U_REQUIRE(lds <= 160 * 1024);
  dim3 grid(nsb, (Nout + CO_BLK - 1) / CO_BLK, NZ), block(256);
  L3U_REQUIRE(NSW == 1);
  const int KSn = K <= 16 ? 4 : (K <= 32 ? 8 : (K <= 64 ? 16 : 0));
#define PWF(NC_, V_, X_, KS_) hipLaunchKernelGGL((pw_fwd_kernel<T, NC_, 1, V_, X_, KS_>), grid, block, lds, \
      stream, x, x_nstride, w, w_layout, bias, y, y_nstride, accumulate, stat_part, K, Nout, S, nsb, \
      Dq, Hq, Wq, p2.x, p2.xns, p2.w, p2.y, p2.yns, p2.stat, N)
#define PWF_K(NC_, V_, X_) do { if (KSn == 4) PWF(NC_, V_, X_, 4); else if (KSn == 8) PWF(NC_, V_, X_, 8); \
                                else if (KSn == 16) PWF(NC_, V_, X_, 16); else PWF(NC_, V_, X_, 0); } while (0)
#define PWF_X(NC_, V_) do { if (xm == 1) PWF_K(NC_, V_, 1); else if (xm == 2) PWF_K(NC_, V_, 2); else PWF_K(NC_, V_, 0); } while (0)
#define PWF_V(NC_) do { if (vec) PWF_X(NC_, true); else PWF_X(NC_, false); } while (0)
  if (NC == 1) PWF_V(1);
  else if (NC == 2) PWF_V(2);
  else PWF_V(4);
#undef PWF_V
#undef PWF_X
#undef PWF_K
#undef PWF
  L3U_CHECK_LAUNCH();
}

template <typename TD, typename TX>
int pw_bwd_weight_launch(const TD* dy, long long dy_nstride, const TX* x, long long x_nstride,
                         float* part, float* bsum, int N, int J, int K, int S, bool gather, int Hq,
                         int Wq, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && J > 0 && K > 0 && S > 0);
  const bool vec = (S % 4 == 0) && (x_nstride % 4 == 0) && (dy_nstride % 4 == 0) &&
                   (!gather || Wq % 4 == 0);
  const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
  int NJ = J <= 16 ? 1 : (J <= 32 ? 2 : 4);
  int NK = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  // shrink the output tile until the grid has enough workgroups to fill the chip
  for (;;) {
    const long long nb = (long long)N * nsc * ((J + 16 * NJ - 1) / (16 * NJ)) *
                         ((K + 16 * NK - 1) / (16 * NK));
    if (nb >= 512 || (NJ == 1 && NK == 1)) break;
    if (NJ >= NK) NJ >>= 1; else NK >>= 1;
  }
  const int ntj = (J + 16 * NJ - 1) / (16 * NJ), ntk = (K + 16 * NK - 1) / (16 * NK);
  const size_t lds = 64 * (size_t)NJ * NK * 4 * sizeof(float);
  dim3 grid(N * nsc, ntj * ntk), block(256);
#define PWB0(A_, B_, V_, G_) hipLaunchKernelGGL((pw_bwd_weight_kernel<TD, TX, A_, B_, V_, G_>), grid, block, lds, \
      stream, dy, dy_nstride, x, x_nstride, part, bsum, J, K, S, SCH, nsc, Hq, Wq)
#define PWB(A_, B_) do { if (gather) { if (vec) PWB0(A_, B_, true, true); else PWB0(A_, B_, false, true); } \
                         else { if (vec) PWB0(A_, B_, true, false); else PWB0(A_, B_, false, false); } } while (0)
  if (NJ == 1 && NK == 1) PWB(1, 1);
  else if (NJ == 1 && NK == 2) PWB(1, 2);
  else if (NJ == 1 && NK == 4) PWB(1, 4);
  else if (NJ == 2 && NK == 1) PWB(2, 1);
  else if (NJ == 2 && NK == 2) PWB(2, 2);
  else if (NJ == 2 && NK == 4) PWB(2, 4);
  else if (NJ == 4 && NK == 1) PWB(4, 1);
  else if (NJ == 4 && NK == 2) PWB(4, 2);
  else PWB(4, 4);
#undef PWB
#undef PWB0
  L3U_CHECK_LAUNCH();
}

constexpr int kConvtPair = 1;   // ConvTranspose3d backward in the x-pair layout (even W) ...
constexpr int kConvtPair1 = 1;   // both pair-layout halves as one launch (convt_pair_bwd_kernel)
// ... for input volumes up to this size (rocprof r2s: at 6^3 35.4 -> 19.8 us; at 24^3 34.3 -> 37.1 us)
constexpr int kConvtPairMaxS = 8192;
constexpr int kCtwMinBlocks = 512;
constexpr int kConvtOnepassAnyw = 0;   // 1: W % 4 != 0 (6^3) by scalar gathers (measured 8 us slower)
constexpr int kConvtOnepassMaxS = 8192;
#ifndef L3U_PWBF_MINBLK
#define L3U_PWBF_MINBLK 512
#endif
// fewest workgroups of a fused pointwise backward (K split in 16-column blocks until reached):
// r5 A/B 512 vs 256 -11.5 us/step (the 24^3 pair goes from 432 to 864 workgroups, dY re-read
// from L2); round 3 measured the opposite on the kernel of then (256 -4 us vs 512)
constexpr int kPwbfMinBlocks = L3U_PWBF_MINBLK;

// wide form: J a multiple of 64 (<= 128), any K; narrow form: J <= 32, K <= 64
constexpr int kPwBwdWide = 1;
bool pw_bwd_wide(int J) { return kPwBwdWide && (J == 64 || J == 128); }
constexpr int kPwbfNkMax = 4;   // K columns per fused-backward workgroup, in 16s
constexpr int kPwwTpbMax = 8;
// 64-voxel tiles per workgroup of pw_bwd_wide_kernel: one at the latency-bound small levels, up
// to kPwwTpbMax on big volumes (fewer weight-gradient partials to write and reduce) while
// each sample keeps >= 32 workgroups per column block
int pww_tpb(int S) {
  const int ntile = (S + 63) / 64;
  int t = 1;
  while (2 * t <= kPwwTpbMax && ntile / (2 * t) >= 32) t *= 2;
  return t;
}
int pww_nblk(int S) { const int t = pww_tpb(S); return ((S + 63) / 64 + t - 1) / t; }

// every pointer aligned to 4 elements of T (one vector load / store)
template <typename T>
bool al4(const void* p) { return ((uintptr_t)p & (4 * sizeof(T) - 1)) == 0; }

template <typename T>
int pw_bwd_tail_impl(const float* dout, long long dout_nstride, const T* out, long long out_nstride,
                     const T* yr, long long yr_nstride, const float* rec, const double* tail_part,
                     int npart, int sel, const T* x, long long x_nstride, const float* w, float* dx,
                     long long dx_nstride, int accumulate, float* part, int N, int J, int K, int S,
                     hipStream_t stream, const float* dscale = nullptr, const float* dpool = nullptr,
                     long long dpns = 0, const unsigned char* pidx = nullptr, int Hf = 0, int Wf = 0) {
  L3U_REQUIRE(N > 0 && l3u_pw_bwd_supported(J, K, S) && !pw_bwd_wide(J));
  L3U_REQUIRE(dpool == nullptr || (pidx && Hf % 2 == 0 && Wf % 4 == 0 && (S / (Hf * Wf)) % 2 == 0 &&
                                   dpns % 2 == 0 && ((uintptr_t)dpool & 7) == 0));
  L3U_REQUIRE(dout && out && yr && rec && tail_part && npart > 0 && (sel == 1 || sel == 2));
  L3U_REQUIRE(x && w && dx && part);
  L3U_REQUIRE(yr_nstride >= 0 || sizeof(T) == 4);   // rank-1 yr: fp32 only
  const bool al = al4<float>(dout) && al4<T>(out) && al4<T>(yr) && al4<T>(x) && al4<float>(dx) &&
                  dout_nstride % 4 == 0 && out_nstride % 4 == 0 && yr_nstride % 4 == 0 &&
                  x_nstride % 4 == 0 && dx_nstride % 4 == 0;
  L3U_REQUIRE(al);
  const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
  const int NJ = J <= 16 ? 1 : 2;
  int NK = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  if (NK > kPwbfNkMax) NK = kPwbfNkMax;
  while (NK > 1 && (long long)N * nsc * ((K + 16 * NK - 1) / (16 * NK)) < kPwbfMinBlocks) NK >>= 1;
  const int nwv = SCH / 64;
  L3U_REQUIRE(nwv >= 1 && nwv <= 8 && SCH == 64 * nwv);
  dim3 grid(N * nsc, (K + 16 * NK - 1) / (16 * NK)), block(64 * nwv);
  const size_t dlds = (size_t)max(nwv, 4) * 16 * kDyTileDS * sizeof(float);   // 16-row dY tiles
#define PWBT1(A_, B_, R_, P_) hipLaunchKernelGGL((pw_bwd_fused_kernel<T, A_, B_, 2, R_, false, P_>), grid, block, \
      dlds, stream, dout, dout_nstride, yr, yr_nstride, rec, tail_part, npart, x, x_nstride, w, dx, dx_nstride, \
      accumulate, part, N, J, K, S, SCH, nsc, out, out_nstride, sel, dscale, dpool, dpns, pidx, Hf, Wf)
#define PWBT0(A_, B_, R_) do { if (dpool) PWBT1(A_, B_, R_, true); else PWBT1(A_, B_, R_, false); } while (0)
#define PWBT(A_, B_) PWBT0(A_, B_, false)
  // a rank-1 yr (the first block's shortcut, K = 1): its own variant
  L3U_REQUIRE(yr_nstride >= 0 || (NJ == 1 && NK == 1));
  if (yr_nstride < 0) { if constexpr (sizeof(T) == 4) PWBT0(1, 1, true); }
  else if (NJ == 1 && NK == 1) PWBT(1, 1);
  else if (NJ == 1 && NK == 2) PWBT(1, 2);
  else if (NJ == 1 && NK == 4) PWBT(1, 4);
  else if (NJ == 2 && NK == 1) PWBT(2, 1);
  else if (NJ == 2 && NK == 2) PWBT(2, 2);
  else PWBT(2, 4);
#undef PWBT
#undef PWBT0
#undef PWBT1
  L3U_CHECK_LAUNCH();
}

// the block tail's two pointwise backwards (conv2.pointwise, sel 1, and the shortcut, sel 2) in one
// launch, grid.z selecting the problem; same dout forms as l3u_pw_bwd_tail[_r1 / _up]
template <typename T>
int pw_bwd_tail_pair_impl(const float* dout, long long dout_nstride, const float* dscale,
                          const float* dpool, long long dpns, const unsigned char* pidx, int Hf,
                          int Wf, const T* out, long long out_nstride, const double* tail_part,
                          int npart, const TailSecond<T>& a, const TailSecond<T>& b, int N, int J,
                          int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && a.K > 0 && b.K > 0 && l3u_pw_bwd_supported(J, a.K, S) &&
              l3u_pw_bwd_supported(J, b.K, S) && !pw_bwd_wide(J));
  L3U_REQUIRE(dpool == nullptr || (pidx && Hf % 2 == 0 && Wf % 4 == 0 && (S / (Hf * Wf)) % 2 == 0 &&
                                   dpns % 2 == 0 && ((uintptr_t)dpool & 7) == 0));
  L3U_REQUIRE(dout && out && tail_part && npart > 0);
  for (const TailSecond<T>* p : {&a, &b}) {
    L3U_REQUIRE(p->yr && p->rec && p->x && p->w && p->dx && p->part && (p->sel == 1 || p->sel == 2));
    L3U_REQUIRE((p->yrns >= 0 || (p == &b && sizeof(T) == 4)) && al4<T>(p->yr) && al4<T>(p->x) && al4<float>(p->dx) && p->yrns % 4 == 0 &&
                p->xns % 4 == 0 && p->dxns % 4 == 0);
  }
  L3U_REQUIRE(al4<float>(dout) && al4<T>(out) && dout_nstride % 4 == 0 && out_nstride % 4 == 0);
  const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
  const int NJ = J <= 16 ? 1 : 2, K = a.K > b.K ? a.K : b.K;
  int NK = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  if (NK > kPwbfNkMax) NK = kPwbfNkMax;
  while (NK > 1 && 2ll * N * nsc * ((K + 16 * NK - 1) / (16 * NK)) < kPwbfMinBlocks) NK >>= 1;
  const int nwv = SCH / 64;
  L3U_REQUIRE(nwv >= 1 && nwv <= 8 && SCH == 64 * nwv);
  dim3 grid(N * nsc, (K + 16 * NK - 1) / (16 * NK), 2), block(64 * nwv);
  const size_t dlds = (size_t)max(nwv, 4) * 16 * kDyTileDS * sizeof(float);   // 16-row dY tiles
#define PWTP1(A_, B_, R_, P_) hipLaunchKernelGGL((pw_bwd_fused_kernel<T, A_, B_, 2, false, R_, P_>), grid, block, \
      dlds, stream, dout, dout_nstride, a.yr, a.yrns, a.rec, tail_part, npart, a.x, a.xns, a.w, a.dx, a.dxns, \
      a.accumulate, a.part, N, J, a.K, S, SCH, nsc, out, out_nstride, a.sel, dscale, dpool, dpns, pidx, \
      Hf, Wf, b)
#define PWTP0(A_, B_, R_) do { if (dpool) PWTP1(A_, B_, R_, true); else PWTP1(A_, B_, R_, false); } while (0)
#define PWTP(A_, B_) PWTP0(A_, B_, false)
  // a rank-1 second operand (the first block's shortcut, K = 1, beside conv2's K = J <= 16)
  L3U_REQUIRE(b.yrns >= 0 || (NJ == 1 && NK == 1));
  if (b.yrns < 0) { if constexpr (sizeof(T) == 4) PWTP0(1, 1, true); }
  else if (NJ == 1 && NK == 1) PWTP(1, 1);
  else if (NJ == 1 && NK == 2) PWTP(1, 2);
  else if (NJ == 1 && NK == 4) PWTP(1, 4);
  else if (NJ == 2 && NK == 1) PWTP(2, 1);
  else if (NJ == 2 && NK == 2) PWTP(2, 2);
  else PWTP(2, 4);
#undef PWTP
#undef PWTP0
#undef PWTP1
  L3U_CHECK_LAUNCH();
}

template <typename T>
int pw_bwd_impl(const float* dy, long long dy_nstride, const T* y, long long y_nstride,
                const float* rec, const double* in_part, int npart, const T* x,
                long long x_nstride, const float* w, float* dx, long long dx_nstride, int accumulate,
                float* part, int N, int J, int K, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && l3u_pw_bwd_supported(J, K, S) && dy && x && w && dx && part);
  L3U_REQUIRE(y == nullptr || (rec && in_part && npart > 0));
  L3U_REQUIRE(y_nstride >= 0 || (sizeof(T) == 4 && y != nullptr && !pw_bwd_wide(J)));   // rank-1 y
  const bool al = al4<float>(dy) && al4<T>(x) && al4<float>(dx) && (dy_nstride % 4 == 0) &&
                  (x_nstride % 4 == 0) && (dx_nstride % 4 == 0) &&
                  (y == nullptr || (al4<T>(y) && y_nstride % 4 == 0));
  L3U_REQUIRE(al);
  if (pw_bwd_wide(J)) {
    dim3 grid(N * pww_nblk(S), (K + 15) / 16), block(256);
#define PWBW(T_, P_) do { if (pww_tpb(S) > 1) hipLaunchKernelGGL((pw_bwd_wide_kernel<T, T_, 4, P_, 0, true>), grid, \
      block, 0, stream, dy, dy_nstride, y, y_nstride, rec, in_part, npart, x, x_nstride, w, dx, dx_nstride, \
      accumulate, part, nullptr, N, J, K, S, 0, 0, pww_tpb(S)); \
      else hipLaunchKernelGGL((pw_bwd_wide_kernel<T, T_, 4, P_, 0>), grid, block, 0, stream, \
      dy, dy_nstride, y, y_nstride, rec, in_part, npart, x, x_nstride, w, dx, dx_nstride, \
      accumulate, part, nullptr, N, J, K, S, 0, 0, 1); } while (0)
    if (J == 64) { if (y) PWBW(1, 1); else PWBW(1, 0); }
    else { if (y) PWBW(2, 1); else PWBW(2, 0); }
#undef PWBW
    L3U_CHECK_LAUNCH();
  }
  const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
  const int NJ = J <= 16 ? 1 : 2;
  // K columns per workgroup: all of them unless the grid would be too small to fill the chip
  int NK = K <= 16 ? 1 : (K <= 32 ? 2 : 4);
  if (NK > kPwbfNkMax) NK = kPwbfNkMax;
  while (NK > 1 && (long long)N * nsc * ((K + 16 * NK - 1) / (16 * NK)) < kPwbfMinBlocks) NK >>= 1;
  const int nwv = SCH / 64;
  L3U_REQUIRE(nwv >= 1 && nwv <= 8 && SCH == 64 * nwv);   // one sweep of the chunk per workgroup
  dim3 grid(N * nsc, (K + 16 * NK - 1) / (16 * NK)), block(64 * nwv);
  const size_t dlds = (size_t)max(nwv, 4) * 16 * kDyTileDS * sizeof(float);   // 16-row dY tiles
  // one input channel with the IN prologue (the first block's conv1.pointwise, y materialised or
  // rank-1): the VALU kernel, same chunks and partial layout
  if (K == 1 && y != nullptr && SCH <= 512 && J <= 32) {
    L3U_REQUIRE(pw_chunk_ok(SCH));   // SCH / 4 threads: whole waves, <= the 128-thread bound
#define PK1(Y_) hipLaunchKernelGGL((pw_bwd_k1_kernel<T, Y_>), dim3(N * nsc), dim3(SCH / 4), 0, stream, dy, \
      dy_nstride, y, y_nstride, rec, in_part, npart, x, x_nstride, w, dx, dx_nstride, accumulate, part, N, J, \
      S, SCH, nsc)
    if (y_nstride < 0) PK1(true); else PK1(false);
#undef PK1
    L3U_CHECK_LAUNCH();
  }
  L3U_REQUIRE(y_nstride >= 0);   // a rank-1 y is K = 1 (above)
#define PWBF(A_, B_) do { if (y) hipLaunchKernelGGL((pw_bwd_fused_kernel<T, A_, B_, 1>), grid, block, dlds, \
      stream, dy, dy_nstride, y, y_nstride, rec, in_part, npart, x, x_nstride, w, dx, dx_nstride, \
      accumulate, part, N, J, K, S, SCH, nsc); \
    else hipLaunchKernelGGL((pw_bwd_fused_kernel<T, A_, B_, 0>), grid, block, dlds, stream, dy, dy_nstride, \
      y, y_nstride, rec, in_part, npart, x, x_nstride, w, dx, dx_nstride, accumulate, part, N, J, K, \
      S, SCH, nsc); } while (0)
  if (NJ == 1 && NK == 1) PWBF(1, 1);
  else if (NJ == 1 && NK == 2) PWBF(1, 2);
  else if (NJ == 1 && NK == 4) PWBF(1, 4);
  else if (NJ == 2 && NK == 1) PWBF(2, 1);
  else if (NJ == 2 && NK == 2) PWBF(2, 2);
  else PWBF(2, 4);
#undef PWBF
  L3U_CHECK_LAUNCH();
}

// two independent plain (PRO 0) wide backwards of the same J, N and S in one launch: a block's
// conv2.pointwise and its Conv1x1 shortcut at the 12^3 / 6^3 levels (both read the block tail's
// dy2 / dr), grid.z selects the problem
template <typename T>
int pw_bwd2_impl(const float* dya, long long dya_nstride, const T* xa, long long xa_nstride,
                 const float* wa, float* dxa, long long dxa_nstride, int acc_a, float* part_a,
                 int Ka, const float* dyb, long long dyb_nstride, const T* xb, long long xb_nstride,
                 const float* wb, float* dxb, long long dxb_nstride, int acc_b, float* part_b,
                 int Kb, int N, int J, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && pw_bwd_wide(J) && Ka > 0 && Kb > 0 && S > 0 && pww_tpb(S) == 1);
  L3U_REQUIRE(dya && xa && wa && dxa && part_a && dyb && xb && wb && dxb && part_b);
  const bool al = al4<float>(dya) && al4<T>(xa) && al4<float>(dxa) && al4<float>(dyb) && al4<T>(xb) &&
                  al4<float>(dxb) && dya_nstride % 4 == 0 && xa_nstride % 4 == 0 &&
                  dxa_nstride % 4 == 0 && dyb_nstride % 4 == 0 && xb_nstride % 4 == 0 &&
                  dxb_nstride % 4 == 0;
  L3U_REQUIRE(al);
  const WideSecond<T> p2{dyb, dyb_nstride, xb, xb_nstride, wb, dxb, dxb_nstride, acc_b, part_b, Kb};
  const int K = Ka > Kb ? Ka : Kb;
  dim3 grid(N * pww_nblk(S), (K + 15) / 16, 2), block(256);
#define PWB2(T_) hipLaunchKernelGGL((pw_bwd_wide_kernel<T, T_, 4, 0, 0>), grid, block, 0, stream, dya, \
      dya_nstride, nullptr, 0, nullptr, nullptr, 0, xa, xa_nstride, wa, dxa, dxa_nstride, acc_a, part_a, \
      nullptr, N, J, Ka, S, 0, 0, 1, p2)
  if (J == 64) PWB2(1);
  else PWB2(2);
#undef PWB2
  L3U_CHECK_LAUNCH();
}

template <typename T>
int convt_bwd_fused_impl(const float* dy, long long dy_nstride, const T* x, long long x_nstride,
                         const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                         int N, int Ci, int Co, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(l3u_convt_bwd_fused_nparts(N, Ci, Co, D, H, W) > 0 && dy && x && w && dx && wpart);
  if (convt_tile_nparts(N, Ci, Co, D, H, W) > 0)   // the one-read tile kernel (convt.hip)
    return convt_tile_launch<T>(dy, dy_nstride, x, x_nstride, w, dx, dx_nstride, wpart, bpart, N, Ci,
                                Co, D, H, W, stream);
  const int S = D * H * W, J = Co * 8;
  const bool vec = W % 4 == 0 && S % 4 == 0 && dy_nstride % 4 == 0 && x_nstride % 4 == 0 &&
                   dx_nstride % 4 == 0 && al4<float>(dy) && al4<T>(x) && al4<float>(dx);
  dim3 grid(N * pww_nblk(S), (Ci + 15) / 16);
#define CTB(T_, NW_, G_) do { if (pww_tpb(S) > 1) hipLaunchKernelGGL((pw_bwd_wide_kernel<T, T_, NW_, 0, G_, true>), \
      grid, dim3(64 * NW_), 0, stream, dy, dy_nstride, nullptr, 0, nullptr, nullptr, 0, x, x_nstride, w, dx, \
      dx_nstride, 0, wpart, bpart, N, J, Ci, S, H, W, pww_tpb(S)); \
      else hipLaunchKernelGGL((pw_bwd_wide_kernel<T, T_, NW_, 0, G_>), grid, dim3(64 * NW_), \
      0, stream, dy, dy_nstride, nullptr, 0, nullptr, nullptr, 0, x, x_nstride, w, dx, dx_nstride, 0, \
      wpart, bpart, N, J, Ci, S, H, W, 1); } while (0)
#define CTB_G(T_, NW_) do { if (vec) CTB(T_, NW_, 1); else CTB(T_, NW_, 2); } while (0)
  if (J == 64) CTB_G(1, 4);
  else if (J == 128) CTB_G(2, 4);
  else if (J == 256) CTB_G(2, 8);
  else CTB_G(2, 16);
#undef CTB_G
#undef CTB
  L3U_CHECK_LAUNCH();
}

template <typename T>
int convt_bwd_impl(const float* dy, long long dy_nstride, const T* x, long long x_nstride,
                   const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                   int N, int Ci, int Co, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Ci > 0 && Co > 0 && D > 0 && H > 0 && W > 0);
  const int S = D * H * W;
  const bool pdx = kConvtPair && S <= kConvtPairMaxS && W % 2 == 0 && dy_nstride % 4 == 0 &&
                   dx_nstride % 2 == 0 && al4<float>(dy) && ((uintptr_t)dx & 7) == 0;
  const bool pdw = kConvtPair && S <= kConvtPairMaxS && W % 2 == 0 && x_nstride % 2 == 0 &&
                   dy_nstride % 4 == 0 && al4<float>(dy) && ((uintptr_t)x & (2 * sizeof(T) - 1)) == 0;
  if (kConvtPair1 && pdx && pdw && Co >= 16) {
    // one launch for both halves (same tile choices as the two launches below)
    const int P = D * H * (W / 2);
    const int NC = Ci % 32 == 0 && (long long)N * ((P + 15) / 16) * (Ci / 32) >= 256 ? 2 : 1;
    const int gx = (P + 15) / 16, gy = (Ci + 16 * NC - 1) / (16 * NC), nA = gx * gy * N;
    const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
    int NJ = Ci % 32 == 0 ? 2 : 1, NG = Co % 16 == 0 ? 4 : (Co % 8 == 0 ? 2 : 1);
    for (;;) {
      const long long nb = (long long)N * nsc * ((Ci + 16 * NJ - 1) / (16 * NJ)) *
                           ((Co + 4 * NG - 1) / (4 * NG));
      if (nb >= kCtwMinBlocks || (NJ == 1 && NG == 1)) break;
      if (NG > 1) NG >>= 1; else NJ >>= 1;
    }
    const int gwx = N * nsc, gwy = ((Ci + 16 * NJ - 1) / (16 * NJ)) * ((Co + 4 * NG - 1) / (4 * NG));
    dim3 grid(nA + gwx * gwy), block(256);
#define CPB(NC_, NJ_, NG_) hipLaunchKernelGGL((convt_pair_bwd_kernel<T, NC_, NJ_, NG_>), grid, block, 0, \
      stream, dy, dy_nstride, w, dx, dx_nstride, x, x_nstride, wpart, bpart, Ci, Co, D, H, W, SCH, nsc, \
      gx, gy, nA, gwx)
#define CPB_G(NC_, NJ_) do { if (NG == 4) CPB(NC_, NJ_, 4); else if (NG == 2) CPB(NC_, NJ_, 2); \
                             else CPB(NC_, NJ_, 1); } while (0)
    if (NC == 2) { if (NJ == 2) CPB_G(2, 2); else CPB_G(2, 1); }
    else { if (NJ == 2) CPB_G(1, 2); else CPB_G(1, 1); }
#undef CPB_G
#undef CPB
    L3U_CHECK_LAUNCH();
  }
  // dX[ci][s] = sum_{co,abc} w[ci][co*8+abc] dY[co][up(s, abc)] (all gradients: fp32): in the
  // x-pair layout for even W (8-byte aligned rows), else the GEMM with X gathered
  int rc;
  if (kConvtPair && S <= kConvtPairMaxS && W % 2 == 0 && dy_nstride % 4 == 0 &&
      dx_nstride % 2 == 0 && al4<float>(dy) &&
      ((uintptr_t)dx & 7) == 0) {
    const int P = D * H * (W / 2);
    const int NC = Ci % 32 == 0 && (long long)N * ((P + 15) / 16) * (Ci / 32) >= 256 ? 2 : 1;
    const int KW = Co >= 16 ? 4 : (Co >= 8 ? 2 : 1);
    dim3 grid((P + 15) / 16, (Ci + 16 * NC - 1) / (16 * NC), N), block(64 * KW);
#define CTP(NC_, KW_) hipLaunchKernelGGL((convt_dx_pair_kernel<NC_, KW_>), grid, block, 0, stream, dy, \
      dy_nstride, w, dx, dx_nstride, Ci, Co, D, H, W)
    if (NC == 2) { if (KW == 4) CTP(2, 4); else if (KW == 2) CTP(2, 2); else CTP(2, 1); }
    else { if (KW == 4) CTP(1, 4); else if (KW == 2) CTP(1, 2); else CTP(1, 1); }
#undef CTP
    rc = (int)hipGetLastError();
  } else {
    rc = pw_launch<float>(dy, dy_nstride, w, 0, nullptr, dx, dx_nstride, 0, nullptr, N, Co * 8, Ci, S,
                          2, D, H, W, stream);
  }
  if (rc != 0) return rc;
  // dW[ci][co*8+abc] = sum_s x[ci][s] dY[co][up(s, abc)] and, in the same launch,
  // db[co] = sum of dY over the up-sampled volume: bpart[N*nsc][Co]
  if (kConvtPair && S <= kConvtPairMaxS && W % 2 == 0 && x_nstride % 2 == 0 &&
      dy_nstride % 4 == 0 && al4<float>(dy) &&
      ((uintptr_t)x & (2 * sizeof(T) - 1)) == 0) {
    const int SCH = pw_sch(S), nsc = (S + SCH - 1) / SCH;
    // as many (ci, co) tiles per workgroup as keep >= kCtwMinBlocks workgroups
    int NJ = Ci % 32 == 0 ? 2 : 1, NG = Co % 16 == 0 ? 4 : (Co % 8 == 0 ? 2 : 1);
    for (;;) {
      const long long nb = (long long)N * nsc * ((Ci + 16 * NJ - 1) / (16 * NJ)) *
                           ((Co + 4 * NG - 1) / (4 * NG));
      if (nb >= kCtwMinBlocks || (NJ == 1 && NG == 1)) break;
      if (NG > 1) NG >>= 1; else NJ >>= 1;
    }
    dim3 grid(N * nsc, ((Ci + 16 * NJ - 1) / (16 * NJ)) * ((Co + 4 * NG - 1) / (4 * NG))), block(256);
#define CTW(NJ_, NG_) hipLaunchKernelGGL((convt_dw_pair_kernel<T, NJ_, NG_>), grid, block, 0, stream, x, \
      x_nstride, dy, dy_nstride, wpart, bpart, Ci, Co, D, H, W, SCH, nsc)
    if (NJ == 2) { if (NG == 4) CTW(2, 4); else if (NG == 2) CTW(2, 2); else CTW(2, 1); }
    else { if (NG == 4) CTW(1, 4); else if (NG == 2) CTW(1, 2); else CTW(1, 1); }
#undef CTW
    L3U_CHECK_LAUNCH();
  }
  return pw_bwd_weight_launch<T, float>(x, x_nstride, dy, dy_nstride, wpart, bpart, N, Ci, Co * 8, S,
                                        true, H, W, stream);
}

template <typename T>
int pw_fwd2_impl(const T* xa, long long xa_nstride, const float* wa, T* ya, long long ya_nstride,
                 float* stat_a, const T* xb, long long xb_nstride, const float* wb, T* yb,
                 long long yb_nstride, float* stat_b, int N, int K, int Nout, int S,
                 hipStream_t stream) {
  L3U_REQUIRE(xa && wa && ya && xb && wb && yb && (stat_a == nullptr) == (stat_b == nullptr));
  L3U_REQUIRE(S % 4 == 0 && xa_nstride % 4 == 0 && ya_nstride % 4 == 0 && xb_nstride % 4 == 0 &&
              yb_nstride % 4 == 0);   // both problems on the vector path
  const PwSecond<T> b{xb, xb_nstride, wb, yb, yb_nstride, stat_b};
  return pw_launch<T>(xa, xa_nstride, wa, 0, nullptr, ya, ya_nstride, 0, stat_a, N, K, Nout, S, 0, 0,
                      0, 0, stream, &b);
}

}  // namespace

extern "C" {

int l3u_pw_stat_nsb(int K, int Nout, int S) {
  if (pw_use_ks(S, K)) return (S + 63) / 64;
  const int CO_BLK = Nout <= 16 ? 16 : (Nout <= 32 ? 32 : 64);
  const int TSB = 256 * pw_nsw(CO_BLK / 16);
  return (S + TSB - 1) / TSB;
}

int l3u_pw_bwd_weight_nparts(int N, int S) {
  const int SCH = pw_sch(S);
  return N * ((S + SCH - 1) / SCH);
}

int l3u_pw_bwd_chunk(int S) { return S > 0 ? pw_sch(S) : 0; }

int l3u_pw_bwd_supported(int J, int K, int S) {
  if (!(J > 0 && K > 0 && S > 0 && S % 4 == 0)) return 0;
  return (pw_bwd_wide(J) || (J <= 32 && K <= 64)) ? 1 : 0;
}

int l3u_pw_bwd2_supported(int J, int S) { return pw_bwd_wide(J) && pww_tpb(S) == 1 ? 1 : 0; }

int l3u_pw_bwd_nparts(int N, int J, int K, int S) {
  if (!l3u_pw_bwd_supported(J, K, S)) return 0;
  return pw_bwd_wide(J) ? N * pww_nblk(S) : l3u_pw_bwd_weight_nparts(N, S);
}

// fused ConvTranspose3d backward: Co*8 = 16 * 2 * NWV rows (Co in {8, 16, 32, 64}).  Offered for
// the mid-size levels only (measured, tools/pwbench.py --convt-only): at 24^3 the three-launch
// path is as fast (the gathered A-layout reads coalesce poorly at that volume) and at 6^3
// (W % 4 != 0: scalar gathers) it is faster.
int l3u_convt_bwd_fused_nparts(int N, int Ci, int Co, int D, int H, int W) {
  const int nt = convt_tile_nparts(N, Ci, Co, D, H, W);
  if (nt > 0) return nt;
  if (!(N > 0 && Ci > 0 && (Co == 8 || Co == 16 || Co == 32 || Co == 64) && D > 0 && H > 0 && W > 0))
    return 0;
  if ((!kConvtOnepassAnyw && W % 4 != 0) || D * H * W > kConvtOnepassMaxS) return 0;
  return N * pww_nblk(D * H * W);
}

}  // extern "C"

// ---- C-ABI: fp32 entry points and their _bf16 twins (include/l3u.h) ----------------------------
#define P_PWF(TT) (const TT* x, long long x_nstride, const float* w, int w_layout,                \
    const float* bias, TT* y, long long y_nstride, int accumulate, float* stat_part, int N, int K,  \
    int Nout, int S, hipStream_t stream)
L3U_TWIN(l3u_pw_fwd, P_PWF, pw_launch(bp(x), x_nstride, w, w_layout, bias, bp(y), y_nstride,
         accumulate, stat_part, N, K, Nout, S, 0, 0, 0, 0, stream))
#define P_PF2(TT) (const TT* xa, long long xa_nstride, const float* wa, TT* ya,                    \
    long long ya_nstride, float* stat_a, const TT* xb, long long xb_nstride, const float* wb,       \
    TT* yb, long long yb_nstride, float* stat_b, int N, int K, int Nout, int S, hipStream_t stream)
L3U_TWIN(l3u_pw_fwd2, P_PF2, pw_fwd2_impl(bp(xa), xa_nstride, wa, bp(ya), ya_nstride, stat_a, bp(xb),
         xb_nstride, wb, bp(yb), yb_nstride, stat_b, N, K, Nout, S, stream))
#define P_CTF(TT) (const TT* x, long long x_nstride, const float* w, const float* bias, TT* out,   \
    long long out_nstride, int N, int Ci, int Co, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_convt_fwd, P_CTF, (D > 0 && H > 0 && W > 0)
         ? pw_launch(bp(x), x_nstride, w, 1, bias, bp(out), out_nstride, 0, nullptr, N, Ci, Co * 8,
                     D * H * W, 1, D, H, W, stream)
         : (int)hipErrorInvalidValue)
#define P_PBW(TT) (const float* dy, long long dy_nstride, const TT* x, long long x_nstride,        \
    float* part, int N, int J, int K, int S, hipStream_t stream)
L3U_TWIN(l3u_pw_bwd_weight, P_PBW, pw_bwd_weight_launch(dy, dy_nstride, bp(x), x_nstride, part,
         nullptr, N, J, K, S, false, 0, 0, stream))
#define P_PBT(TT) (const float* dout, long long dout_nstride, const TT* out, long long out_nstride, \
    const TT* yr, long long yr_nstride, const float* rec, const double* tail_part, int npart,        \
    int sel, const TT* x, long long x_nstride, const float* w, float* dx, long long dx_nstride,     \
    int accumulate, float* part, int N, int J, int K, int S, hipStream_t stream)
L3U_TWIN(l3u_pw_bwd_tail, P_PBT, pw_bwd_tail_impl(dout, dout_nstride, bp(out), out_nstride, bp(yr),
         yr_nstride, rec, tail_part, npart, sel, bp(x), x_nstride, w, dx, dx_nstride, accumulate,
         part, N, J, K, S, stream))
// rank-1 block-output gradient dout[j] = dscale[j] * dz (dz one channel, l3u_outconv_bwd_dz)
#define P_PBT1(TT) (const float* dz, long long dz_nstride, const float* dscale, const TT* out,        \
    long long out_nstride, const TT* yr, long long yr_nstride, const float* rec,                     \
    const double* tail_part, int npart, int sel, const TT* x, long long x_nstride, const float* w,   \
    float* dx, long long dx_nstride, int accumulate, float* part, int N, int J, int K, int S,        \
    hipStream_t stream)
// the block-output gradient = skip gradient + the next level's MaxPool3d backward, folded in
#define P_PBTU(TT) (const float* dskip, long long dskip_nstride, const float* dpool,                  \
    long long dpool_nstride, const unsigned char* idx, const TT* out, long long out_nstride,         \
    const TT* yr, long long yr_nstride, const float* rec, const double* tail_part, int npart,         \
    int sel, const TT* x, long long x_nstride, const float* w, float* dx, long long dx_nstride,     \
    int accumulate, float* part, int N, int J, int K, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_pw_bwd_tail_up, P_PBTU, dpool == nullptr ? (int)hipErrorInvalidValue :
         pw_bwd_tail_impl(dskip, dskip_nstride, bp(out), out_nstride, bp(yr), yr_nstride, rec, tail_part,
         npart, sel, bp(x), x_nstride, w, dx, dx_nstride, accumulate, part, N, J, K, D * H * W, stream,
         nullptr, dpool, dpool_nstride, idx, H, W))
L3U_TWIN(l3u_pw_bwd_tail_r1, P_PBT1, dscale == nullptr ? (int)hipErrorInvalidValue :
         pw_bwd_tail_impl(dz, dz_nstride, bp(out), out_nstride, bp(yr), yr_nstride, rec, tail_part,
         npart, sel, bp(x), x_nstride, w, dx, dx_nstride, accumulate, part, N, J, K, S, stream, dscale))
// the block tail's conv2.pointwise (sel 1) and shortcut (sel 2) backwards in one launch; dscale /
// dpool (+ idx, Hf, Wf) as l3u_pw_bwd_tail_r1 / _up, or NULL
#define P_PBTP(TT) (const float* dout, long long dout_nstride, const float* dscale,                   \
    const float* dpool, long long dpool_nstride, const unsigned char* idx, int Hf, int Wf,          \
    const TT* out, long long out_nstride, const double* tail_part, int npart, const TT* yra,         \
    long long yra_nstride, const float* reca, const TT* xa, long long xa_nstride, const float* wa,   \
    float* dxa, long long dxa_nstride, int acc_a, float* part_a, int Ka, int sel_a, const TT* yrb,   \
    long long yrb_nstride, const float* recb, const TT* xb, long long xb_nstride, const float* wb,   \
    float* dxb, long long dxb_nstride, int acc_b, float* part_b, int Kb, int sel_b, int N, int J,    \
    int S, hipStream_t stream)
L3U_TWIN(l3u_pw_bwd_tail_pair, P_PBTP, pw_bwd_tail_pair_impl(dout, dout_nstride, dscale, dpool,
         dpool_nstride, idx, Hf, Wf, bp(out), out_nstride, tail_part, npart,
         TailSecond<std::remove_const_t<std::remove_pointer_t<decltype(bp(out))>>>{bp(yra), yra_nstride,
             reca, bp(xa), xa_nstride, wa, dxa, dxa_nstride, acc_a, part_a, Ka, sel_a},
         TailSecond<std::remove_const_t<std::remove_pointer_t<decltype(bp(out))>>>{bp(yrb), yrb_nstride,
             recb, bp(xb), xb_nstride, wb, dxb, dxb_nstride, acc_b, part_b, Kb, sel_b},
         N, J, S, stream))
#define P_PBD(TT) (const float* dy, long long dy_nstride, const TT* y, long long y_nstride,         \
    const float* rec, const double* in_part, int npart, const TT* x, long long x_nstride,           \
    const float* w, float* dx, long long dx_nstride, int accumulate, float* part, int N, int J,     \
    int K, int S, hipStream_t stream)
L3U_TWIN(l3u_pw_bwd, P_PBD, pw_bwd_impl(dy, dy_nstride, bp(y), y_nstride, rec, in_part, npart,
         bp(x), x_nstride, w, dx, dx_nstride, accumulate, part, N, J, K, S, stream))
#define P_PB2(TT) (const float* dya, long long dya_nstride, const TT* xa, long long xa_nstride,     \
    const float* wa, float* dxa, long long dxa_nstride, int acc_a, float* part_a, int Ka,           \
    const float* dyb, long long dyb_nstride, const TT* xb, long long xb_nstride, const float* wb,  \
    float* dxb, long long dxb_nstride, int acc_b, float* part_b, int Kb, int N, int J, int S,      \
    hipStream_t stream)
L3U_TWIN(l3u_pw_bwd2, P_PB2, pw_bwd2_impl(dya, dya_nstride, bp(xa), xa_nstride, wa, dxa, dxa_nstride,
         acc_a, part_a, Ka, dyb, dyb_nstride, bp(xb), xb_nstride, wb, dxb, dxb_nstride, acc_b, part_b,
         Kb, N, J, S, stream))
#define P_CBF(TT) (const float* dy, long long dy_nstride, const TT* x, long long x_nstride,         \
    const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart, int N, int Ci,     \
    int Co, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_convt_bwd_fused, P_CBF, convt_bwd_fused_impl(dy, dy_nstride, bp(x), x_nstride, w,
         dx, dx_nstride, wpart, bpart, N, Ci, Co, D, H, W, stream))
L3U_TWIN(l3u_convt_bwd, P_CBF, convt_bwd_impl(dy, dy_nstride, bp(x), x_nstride, w, dx,
         dx_nstride, wpart, bpart, N, Ci, Co, D, H, W, stream))
