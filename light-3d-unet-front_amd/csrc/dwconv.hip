// Depthwise 3x3x3 convolution (stride 1, zero padding 1, no bias) — forward and fused backward.
// Replaces nn.Conv3d(C, C, 3, 1, 1, groups=C, bias=False)   light_unet/models/unet3d.py:16-17.
//
// Mapping: one 256-thread workgroup owns one (n, c) channel volume and a slab of
// TZ output z-planes.  It walks the input planes z0-1 .. z0+TZ once ("2.5D" blocking): each plane
// is loaded coalesced (W contiguous) into a zero-haloed (H+2)x(W+2) LDS image, and each thread
// applies the 3 kernel slices of its (y, x) positions to 3 rolling register accumulators, so
// every input element is read from HBM once per slab and from LDS 9 times.  Next-plane global
// loads are issued before the current plane's stencil (register prefetch) so HBM latency hides
// under LDS/VALU work.  Logical workgroup ids are XCD-remapped so that slabs of one channel that
// share halo planes run on the same XCD (shared L2).
//
// MODE 1 fuses the InstanceNorm-apply + LeakyReLU + Dropout3d transform of the previous layer
// (unet3d.py:84-88) into the input load: a = lrelu(scale*y + shift), with zero padding applied in
// the transformed domain (as the reference pads the conv input a).
#include <type_traits>
#include <utility>

#include "common.h"
using namespace l3u;

namespace {

template <typename T, int MODE, int P>
__global__ __launch_bounds__(256) void dw3_fwd_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    const float* __restrict__ rec, l3u_norm_src src, int has_src, T* __restrict__ y,
    long long yns, int C, int D, int H, int W, int TZ, int nchunk) {
  L3U_STAMP_SCOPE(201);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int HW = H * W, PW = W + 2, PP = (H + 2) * PW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lb % nchunk;
  const int nc = lb / nchunk;
  const int c = nc % C, n = nc / C;
  const int z0 = chunk * TZ, z1 = min(z0 + TZ, D);
  const T* xp = x + (long long)n * xns + (long long)c * D * HW;
  T* yp = y + (long long)n * yns + (long long)c * D * HW;
  const int tid = threadIdx.x;

  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + t];
  float sc = 1.f, sh = 0.f, mu = 0.f;
  if (MODE == 1) {
    if (has_src) {
      float* s8 = lds + 2 * PP;
      block_record(src, n, c, C, chunk == 0, s8);
      mu = s8[0]; sc = s8[2]; sh = s8[3];
    } else {
      mu = rec[(long long)nc * kRec + 0];
      sc = rec[(long long)nc * kRec + 2];
      sh = rec[(long long)nc * kRec + 3];
    }
  }
  for (int i = tid; i < 2 * PP; i += 256) lds[i] = 0.f;

  int lbase[P];
  bool own[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int p = tid + k * 256;
    own[k] = p < HW;
    const int yy = p / W, xx = p - yy * W;
    lbase[k] = own[k] ? (yy + 1) * PW + xx + 1 : 0;
  }
  float a0[P], a1[P], a2[P], nxt[P];
#pragma unroll
  for (int k = 0; k < P; ++k) { a0[k] = a1[k] = a2[k] = 0.f; nxt[k] = 0.f; }

  // prologue: fetch plane z0-1
  {
    const int zi = z0 - 1;
    if (zi >= 0) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) nxt[k] = ld1(xp + (long long)zi * HW + tid + k * 256);
    }
  }
  __syncthreads();
  for (int zi = z0 - 1; zi <= z1; ++zi) {
    float* buf = lds + ((zi - z0 + 1) & 1) * PP;
    const bool in = zi >= 0 && zi < D;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (own[k]) {
        float v = nxt[k];
        if (MODE == 1) v = lrelu(fmaf(sc, v - mu, sh));
        buf[lbase[k]] = in ? v : 0.f;
      }
    }
    // prefetch the next plane while this one is consumed
    const int zn = zi + 1;
    if (zn <= z1 && zn < D) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) nxt[k] = ld1(xp + (long long)zn * HW + tid + k * 256);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (!own[k]) continue;
      const float* b = buf + lbase[k];
      float v[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) v[dy * 3 + dx] = b[(dy - 1) * PW + (dx - 1)];
      // input plane zi feeds output plane zi+1 with slice kd=0, zi with kd=1, zi-1 with kd=2
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        a2[k] = fmaf(wk[j], v[j], a2[k]);
        a1[k] = fmaf(wk[9 + j], v[j], a1[k]);
        a0[k] = fmaf(wk[18 + j], v[j], a0[k]);
      }
    }
    const int zo = zi - 1;
    if (zo >= z0 && zo < z1) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) st1(yp + (long long)zo * HW + tid + k * 256, a0[k]);
    }
#pragma unroll
    for (int k = 0; k < P; ++k) { a0[k] = a1[k]; a1[k] = a2[k]; a2[k] = 0.f; }
  }
}

// Fused backward: dA = conv^T(dZ) (data gradient, flipped stencil) and dW = sum dZ (x) A (27 taps)
// in ONE pass over dZ and A.  Step s loads dZ plane zd = z0-1+s and A plane za = zd-1; the thread
// keeps its own dZ values of planes zd-2..zd in registers so each A-neighbourhood read from LDS
// feeds all three kernel depths.  dW is owned by the dZ plane (zd in [z0, z1)), so every product
// is counted exactly once across slabs.  Partial dW per workgroup -> dw_part[c][n*nchunk+chunk][27]
// (deterministic second stage: l3u_reduce_segments).
// MODE 1: A = lrelu(scale*y + shift) recomputed from y; the kernel emits
// dpre = dA * k * lrelu'(pre) (gradient at the InstanceNorm output before the activation) and the
// per-(n,c) partial sums  sum(dpre), sum(dpre * xhat)  for the InstanceNorm backward.
template <typename T, int MODE, int P>
__global__ __launch_bounds__(256) void dw3_bwd_kernel(
    const float* __restrict__ dz, long long dzns, const T* __restrict__ x, long long xns,
    const float* __restrict__ w, const float* __restrict__ rec, float* __restrict__ dx,
    long long dxns, int accumulate, float* __restrict__ dw_part, double* __restrict__ in_part,
    int N, int C, int D, int H, int W, int TZ, int nchunk) {
  L3U_STAMP_SCOPE(202);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int HW = H * W, PW = W + 2, PP = (H + 2) * PW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lb % nchunk;
  const int nc = lb / nchunk;
  const int c = nc % C, n = nc / C;
  const int z0 = chunk * TZ, z1 = min(z0 + TZ, D);
  const long long cofs = (long long)c * D * HW;
  const float* dzp = dz + (long long)n * dzns + cofs;
  const T* xp = x + (long long)n * xns + cofs;
  float* dxp = dx + (long long)n * dxns + cofs;
  const int tid = threadIdx.x;
  float* dzb = lds;            // 2 planes
  float* ab = lds + 2 * PP;    // 2 planes

  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + t];
  float sc = 1.f, sh = 0.f, kk = 1.f, mean = 0.f, rstd = 1.f;
  if (MODE == 1) {
    const float* r = rec + (long long)nc * kRec;
    mean = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4];
  }
  for (int i = tid; i < 4 * PP; i += 256) lds[i] = 0.f;

  int lbase[P];
  bool own[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int p = tid + k * 256;
    own[k] = p < HW;
    const int yy = p / W, xx = p - yy * W;
    lbase[k] = own[k] ? (yy + 1) * PW + xx + 1 : 0;
  }
  float d0[P], d1[P], d2[P];       // dA rolling accumulators for planes zd-1, zd, zd+1
  float g0[P], g1[P], g2[P];       // own dZ of planes zd-2, zd-1, zd (zero when not owned)
#pragma unroll
  for (int k = 0; k < P; ++k) d0[k] = d1[k] = d2[k] = g0[k] = g1[k] = g2[k] = 0.f;
  float gw[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) gw[t] = 0.f;
  double s1 = 0.0, s2 = 0.0;

  const int zlo = max(0, z0 - 1), zhi = min(D - 1, z1);   // planes that carry data
  const int nsteps = z1 - z0 + 3;
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int zd = z0 - 1 + s, za = zd - 1;
    float* dbuf = dzb + (s & 1) * PP;
    float* abuf = ab + (s & 1) * PP;
    const bool ldz = zd >= zlo && zd <= zhi;
    const bool la = za >= zlo && za <= zhi;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (own[k]) {
        const long long off = tid + k * 256;
        dbuf[lbase[k]] = ldz ? ld1(dzp + (long long)zd * HW + off) : 0.f;
        float v = 0.f;
        if (la) {
          v = ld1(xp + (long long)za * HW + off);
          if (MODE == 1) v = lrelu(fmaf(sc, v - mean, sh));
        }
        abuf[lbase[k]] = v;
      }
    }
    __syncthreads();
    const bool zd_owned = zd >= z0 && zd < z1;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (!own[k]) continue;
      // dA: flipped stencil of dZ plane zd into dA planes zd-1 (kd=0), zd (kd=1), zd+1 (kd=2)
      const float* b = dbuf + lbase[k];
      float v[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx) v[dy * 3 + dxx] = b[(dy - 1) * PW + (dxx - 1)];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        d0[k] = fmaf(wk[8 - j], v[j], d0[k]);
        d1[k] = fmaf(wk[17 - j], v[j], d1[k]);
        d2[k] = fmaf(wk[26 - j], v[j], d2[k]);
      }
      g0[k] = g1[k];
      g1[k] = g2[k];
      g2[k] = zd_owned ? v[4] : 0.f;
      // dW: A plane za pairs with dZ planes za+1 (kd=0 -> g2), za (kd=1 -> g1), za-1 (kd=2 -> g0)
      const float* a = abuf + lbase[k];
      float u[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx) u[dy * 3 + dxx] = a[(dy - 1) * PW + (dxx - 1)];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        gw[j] = fmaf(g2[k], u[j], gw[j]);
        gw[9 + j] = fmaf(g1[k], u[j], gw[9 + j]);
        gw[18 + j] = fmaf(g0[k], u[j], gw[18 + j]);
      }
    }
    const int zf = zd - 1;   // dA plane zf is complete
    if (dx != nullptr && zf >= z0 && zf < z1) {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        if (!own[k]) continue;
        const long long idx = (long long)zf * HW + tid + k * 256;
        if (MODE == 1) {
          const float yv = ld1(xp + idx);
          const float pre = fmaf(sc, yv - mean, sh);
          const float dp = d0[k] * kk * lrelu_d(pre);
          const float xh = (yv - mean) * rstd;
          st1(dxp + idx, dp);
          s1 += dp;
          s2 += (double)dp * xh;
        } else {
          st1(dxp + idx, accumulate ? ld1(dxp + idx) + d0[k] : d0[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) { d0[k] = d1[k]; d1[k] = d2[k]; d2[k] = 0.f; }
  }
  // workgroup reduction of the 27 weight-gradient taps (+2 fp64 IN sums), fixed order
  __syncthreads();
  float* red = lds;                                        // [4 waves][27]
  double* redd = reinterpret_cast<double*>(lds + 112);     // [4 waves][2]
  const int wv = tid >> 6, ln = tid & 63;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    const float r = wave_sum(gw[t]);
    if (ln == 0) red[wv * 27 + t] = r;
  }
  if (MODE == 1) {
    const double r1 = wave_sum_d(s1), r2 = wave_sum_d(s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
  }
  __syncthreads();
  if (tid < 27 && dw_part != nullptr) {
    const float r = (red[tid] + red[27 + tid]) + (red[54 + tid] + red[81 + tid]);
    dw_part[((long long)c * N * nchunk + (long long)n * nchunk + chunk) * 27 + tid] = r;
  }
  if (MODE == 1 && dx != nullptr && tid >= 32 && tid < 34) {
    const int j = tid - 32;
    const double r = (redd[j] + redd[2 + j]) + (redd[4 + j] + redd[6 + j]);
    // in_part layout [c][n][chunk][2]
    in_part[(((long long)c * N + n) * nchunk + chunk) * 2 + j] = r;
  }
}

int pick_tz(int D) { return D <= 8 ? D : 4; }

// ------------------------------------------------------------------------------------------------
// x-quad variants (W % 4 == 0, 4 <= W <= 256: every production shape).  A workgroup owns
// (n, c, TZ z-planes, RB rows); a thread owns 4 consecutive x of one row and each wave owns RPW
// WHOLE rows (RPW = 64 / (W/4)).  Global traffic is float4 per lane (one 16-B load per input
// quad per plane, one 16-B store per output quad).  The LDS plane image is unpadded
// [RB+2 rows][W]: the quad of each row is one conflict-free ds_read_b128 (a wave's lanes read
// contiguous 16-B slots), and the x-neighbours of a quad come from the adjacent lanes through
// DPP wave shifts (zero at row ends = the conv's zero padding) instead of 4-way bank-conflicted
// 4-byte LDS reads.  Planes outside the volume are committed as zeros, so the stencil never
// branches on z; input planes are staged through registers PD steps ahead of their use.
// ------------------------------------------------------------------------------------------------
// Tuning constants, each the fastest measured value (tools/kbench.py, step A/B; the rejected
// alternatives are listed in profiles/NOTES.md):
constexpr int kDwqPd = 2;          // register prefetch depth (planes in flight), quad forward stencil
constexpr int kDwNwMin = 1;        // fewest waves per workgroup of the quad kernels
constexpr int kTz16MinD = 48;      // 16-plane z slabs from this depth on
constexpr int kDwMinBlocks = 1024; // thinner z slabs until the grid has this many workgroups

struct QGeom {
  int WQ, RPW, NW, RB, ny, TZ, nz, threads;
};

// rows per block: the wave count (1..4) that wastes the fewest row slots over ny strips
QGeom qgeom(int N, int C, int D, int H, int W) {
  QGeom g;
  g.WQ = W / 4;
  g.RPW = 64 / g.WQ;
  int best = 1;
  double beff = -1.0;
  for (int nw = 1; nw <= 4; ++nw) {
    if ((nw - 1) * g.RPW >= H) break;   // a wave with no row at all
    if (nw < kDwNwMin && nw * g.RPW < H) continue;
    const int rb = nw * g.RPW, ny = (H + rb - 1) / rb;
    const double eff = (double)H / (ny * rb);
    if (eff > beff + 1e-9) { beff = eff; best = nw; }
  }
  g.NW = best;
  g.RB = best * g.RPW;
  g.ny = (H + g.RB - 1) / g.RB;
  g.threads = 64 * best;
  g.TZ = D >= kTz16MinD ? 16 : (D >= 32 ? 8 : (D > 8 ? 4 : 8));   // compile-time in the kernels
  while (g.TZ > 2 && (long long)N * C * g.ny * ((D + g.TZ - 1) / g.TZ) < kDwMinBlocks) g.TZ >>= 1;   // {16, 8, 4, 2}
  // 12-plane slabs where 16-plane ones leave under two tiles per SIMD (the 48^3 IN-fused
  // backward of the 16-channel blocks: 1920 -> 2560 one-wave tiles, -8 us/step A/B)
  if (g.TZ == 16 && (long long)N * C * g.ny * ((D + 15) / 16) < 2 * kDwMinBlocks) g.TZ = 12;
  g.nz = (D + g.TZ - 1) / g.TZ;
  return g;
}


bool use_quads(int H, int W) {
  if (W % 4 != 0 || W < 4 || W > 256 || H < 1) return false;
  const QGeom g = qgeom(1, 1, 1, H, W);
  return (g.RB + 2) * g.WQ <= 2 * g.threads;   // register staging: <= 2 quads per thread
}

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

L3U_DEV f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

L3U_DEV float lane_prev(float v) {   // value of lane l-1 (DPP wave_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
L3U_DEV float lane_next(float v) {   // value of lane l+1 (DPP wave_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

// block decode shared by both quad kernels
struct QBlock {
  int n, c, nc, z0, z1, y0, rows, oy, ox, ck;
  bool own, el, er;
};

L3U_DEV QBlock q_decode(int C, int D, int H, int RB, int RPW, int ny, int TZ, int nz, int WQ) {
  QBlock b;
  int t = xcd_remap(blockIdx.x, gridDim.x);
  b.ck = t % (ny * nz);
  const int yb = t % ny; t /= ny;
  const int zb = t % nz; t /= nz;
  b.nc = t;
  b.c = t % C;
  b.n = t / C;
  b.z0 = zb * TZ;
  b.z1 = min(b.z0 + TZ, D);
  b.y0 = yb * RB;
  b.rows = min(RB, H - b.y0);
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int lr = ln / WQ, qx = ln - lr * WQ;
  const int oy = wv * RPW + lr;
  b.own = lr < RPW && oy < b.rows;
  b.oy = b.own ? oy : 0;     // idle lanes read a valid row and never store
  b.ox = qx * 4;
  b.el = qx == 0;
  b.er = qx == WQ - 1;
  return b;
}

// the 6 values around the quad of LDS row `row`: v[0] = x-1 .. v[5] = x+4.  Every lane of the
// wave must execute this (DPP reads the neighbouring lanes).
L3U_DEV void q_nbr(const float* plane, int row, int W, int ox, bool el, bool er, float v[6]) {
  const f4 m = *reinterpret_cast<const f4*>(plane + row * W + ox);
  const float l = lane_prev(m[3]), r = lane_next(m[0]);
  v[0] = el ? 0.f : l;
  v[1] = m[0]; v[2] = m[1]; v[3] = m[2]; v[4] = m[3];
  v[5] = er ? 0.f : r;
}

// Register-staged plane loads (issued early, committed to LDS when their step comes up); held
// in the storage type (bf16 staging costs half the VGPRs) and widened at commit.
template <typename T> struct Raw4 { typedef f4 type; };
template <> struct Raw4<bf16> { typedef b4_t type; };
L3U_DEV f4 widen(f4 v) { return v; }
L3U_DEV f4 widen(b4_t v) { return __builtin_convertvector(v, f4); }
template <typename T>
struct QPre {
  typename Raw4<T>::type v[2];
};

// Per-thread staging map, computed once: global offset (within a plane) and LDS offset of the
// thread's <= 2 quads.  Loads are issued UNCONDITIONALLY from clamped, always-valid addresses
// (branch-free straight-line loads let the compiler count vmcnt exactly instead of draining
// the whole pipeline with vmcnt(0)); the validity mask is applied at commit.  LDS rows outside
// the volume (y = -1, y = H) are never written and stay zero.
struct QMap {
  int goff[2], loff[2];
  bool ok[2];
};

L3U_DEV QMap q_map(int y0, int rows, int H, int W, int WQ, int lpitch = 0, int lofs = 0) {
  QMap m;
  if (lpitch == 0) lpitch = W;
  const int nq = (rows + 2) * WQ;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + k * blockDim.x;
    const int qc = q < nq ? q : 0;
    const int lr = qc / WQ, x = (qc - lr * WQ) * 4, y = y0 - 1 + lr;
    m.ok[k] = q < nq && y >= 0 && y < H;
    m.goff[k] = min(max(y, 0), H - 1) * W + x;
    m.loff[k] = lr * lpitch + lofs + x;
  }
  return m;
}

template <typename T>
L3U_DEV void q_fetch(QPre<T>& p, const T* plane, const QMap& m) {
#pragma unroll
  for (int k = 0; k < 2; ++k) p.v[k] = *reinterpret_cast<const typename Raw4<T>::type*>(plane + m.goff[k]);
}

// commit a staged plane to LDS (zeros for a plane outside the needed z range)
template <bool XF, typename T>
L3U_DEV void q_commit(const QPre<T>& p, float* lplane, const QMap& m, bool in, float sc, float mu,
                      float sh) {
  // out of range: XF folds the zero into the transform (lrelu(0*(v-mu) + 0) = 0), plain
  // planes multiply by 0 (two v_pk_mul per quad instead of four selects)
  const float keep = in ? 1.f : 0.f;
  sc *= keep;
  sh *= keep;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    f4 v = widen(p.v[k]);
    if (XF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = lrelu(fmaf(sc, v[i] - mu, sh));
    } else {
      v *= keep;
    }
    if (m.ok[k]) *reinterpret_cast<f4*>(lplane + m.loff[k]) = v;
  }
}

// keeps a value materialised at this point of the step (see the bwd kernel)
template <typename T>
L3U_DEV void pin(T& v) { asm volatile("" : "+v"(v)); }

// One pass of the 27-tap stencil over a (n, c, slab, strip) tile, input plane by input plane.
//   XF  = 1: the input is transformed on load, a = lrelu(scale*(x-mean)+shift) (IN1 + LeakyReLU
//            + Dropout3d before conv2.depthwise); the record is finalized in-kernel when has_src
//   EPI = 0: forward, y = conv(x)
//   EPI = 1: backward data of the IN-fused conv2: the stencil runs with the FLIPPED taps over dZ
//            (conv^T), and the epilogue emits dpre = dA * k * lrelu'(pre), pre = scale*(ep-mean)
//            + shift (ep = the saved pre-IN activation), plus the fp64 IN-backward sums
//            in_part[c][n][chunk] = {sum dpre, sum dpre*xhat}
//   EPI = 2: backward data, y += conv^T(x)      EPI = 3: backward data, y = conv^T(x)
template <typename T, typename TE, int XF, int EPI, int TZC, int PD = 2>
__global__ __launch_bounds__(256) void dw3q_fwd_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    const float* __restrict__ rec, l3u_norm_src src, int has_src, T* __restrict__ y,
    long long yns, const TE* __restrict__ ep, long long epns, double* __restrict__ in_part,
    int N, int C, int D, int H, int W, int RB, int RPW, int ny, int TZ, int nz) {
  L3U_STAMP_SCOPE(203);
  constexpr bool FLIP = EPI != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int WQ = W >> 2, PP = (RB + 2) * W, HW = H * W;
  const QBlock b = q_decode(C, D, H, RB, RPW, ny, TZ, nz, WQ);
  const long long cofs = (long long)b.c * D * HW;
  const T* xp = x + (long long)b.n * xns + cofs;
  T* yp = y + (long long)b.n * yns + cofs;
  const TE* epp = (EPI == 1 || EPI == 2) ? ep + (long long)b.n * epns + cofs : nullptr;
  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[b.c * 27 + (FLIP ? 26 - t : t)];
  const int zlo = max(0, b.z0 - 1), zhi = min(D - 1, b.z1);
  const QMap qm = q_map(b.y0, b.rows, H, W, WQ);
  auto zc = [&](int z) { return (long long)min(max(z, zlo), zhi) * HW; };   // loads always issue
  const long long qofs = (long long)(b.y0 + b.oy) * W + b.ox;
  // step t consumes input plane zi = z0-1+t; the step count is a compile-time constant and the
  // loop is fully unrolled, so the two staged registers never move (no back-edge copies that
  // would force a vmcnt(0) drain of the pipeline).  The first two planes are requested before
  // the InstanceNorm record is finalized (its partial-sum loads then overlap them).
  QPre<T> pf[PD];   // PD planes in flight (register staging depth)
#pragma unroll
  for (int i = 0; i < PD; ++i) q_fetch(pf[i], xp + zc(b.z0 - 1 + i), qm);
  float sc = 1.f, sh = 0.f, mu = 0.f, rstd = 1.f, kk = 1.f;
  if (XF || EPI == 1) {
    if (has_src) {
      float* s8 = lds + 2 * PP;
      block_record(src, b.n, b.c, C, b.ck == 0, s8);
      mu = s8[0]; rstd = s8[1]; sc = s8[2]; sh = s8[3]; kk = s8[4];
    } else {
      const float* r = rec + (long long)b.nc * kRec;
      mu = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4];
    }
  }
  for (int i = threadIdx.x; i < 2 * PP; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0;
  float s1 = 0.f, s2 = 0.f;   // per-thread sums over <= 4*TZ voxels; widened to fp64 per block
  auto step = [&](int t, QPre<T>& pre) {
    const int zi = b.z0 - 1 + t;
    float* buf = lds + (t & 1) * PP;
    q_commit<XF == 1>(pre, buf, qm, zi >= zlo && zi <= zhi, sc, mu, sh);
    q_fetch(pre, xp + zc(zi + PD), qm);
    const int zo = zi - 1;   // output plane zo has all three input planes after this step
    f4 e = {0.f, 0.f, 0.f, 0.f};
    if (EPI == 1 || EPI == 2) e = ldv4(epp + (long long)min(max(zo, 0), D - 1) * HW + qofs);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float v[6];
      q_nbr(buf, b.oy + r, W, b.ox, b.el, b.er, v);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float w0 = wk[r * 3 + dx], w1 = wk[9 + r * 3 + dx], w2 = wk[18 + r * 3 + dx];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a2[i] = fmaf(w0, v[i + dx], a2[i]);   // input plane zi -> output zi+1 (kd=0)
          a1[i] = fmaf(w1, v[i + dx], a1[i]);   //                -> output zi   (kd=1)
          a0[i] = fmaf(w2, v[i + dx], a0[i]);   //                -> output zi-1 (kd=2)
        }
      }
    }
    pin(a1);
    pin(a2);
    const bool fin = b.own && zo >= b.z0 && zo < b.z1;
    f4 o = a0;
    if (EPI == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pre = fmaf(sc, e[i] - mu, sh);
        const float dp = o[i] * kk * lrelu_d(pre);
        o[i] = dp;
        s1 += fin ? dp : 0.f;
        s2 += fin ? dp * ((e[i] - mu) * rstd) : 0.f;
      }
    } else if (EPI == 2) {
      o += e;
    }
    if (fin) stv4(yp + (long long)zo * HW + qofs, o);
    a0 = a1;
    a1 = a2;
    a2 = f4{0.f, 0.f, 0.f, 0.f};
  };
#pragma unroll
  for (int t = 0; t < TZC + 2; t += PD) {
#pragma unroll
    for (int i = 0; i < PD; ++i)
      if (t + i < TZC + 2) step(t + i, pf[i]);
  }
  if (EPI == 1) {   // fixed-order block reduction of the IN-backward sums
    __syncthreads();
    double* redd = reinterpret_cast<double*>(lds);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, nw = blockDim.x >> 6;
    const double r1 = wave_sum_d((double)s1), r2 = wave_sum_d((double)s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
    __syncthreads();
    if (threadIdx.x < 2) {
      double r = 0.0;
      for (int k = 0; k < nw; ++k) r += redd[k * 2 + threadIdx.x];
      in_part[(((long long)b.c * N + b.n) * (nz * ny) + b.ck) * 2 + threadIdx.x] = r;
    }
  }
}

// Depthwise weight gradient alone: dw_part[c][n*nchunk + chunk][27] = sum over the tile's voxels
// of dZ(v) * A(v + tap), A = x (XF = 0) or lrelu(scale*(x-mean)+shift) (XF = 1).  The A planes go
// through LDS (x-neighbours by DPP); each thread's own dZ quad comes straight from global memory,
// three planes kept in registers.  Split from the data gradient (which is the forward kernel with
// flipped taps) so that each pass keeps few registers and a short VALU chain per byte.
template <typename T, int XF, int TZC>
__global__ __launch_bounds__(256) void dw3q_dw_kernel(
    const float* __restrict__ dz, long long dzns, const T* __restrict__ x, long long xns,
    const float* __restrict__ rec, float* __restrict__ dw_part, int N, int C, int D, int H, int W,
    int RB, int RPW, int ny, int TZ, int nz) {
  L3U_STAMP_SCOPE(204);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int WQ = W >> 2, PP = (RB + 2) * W, HW = H * W;
  const QBlock b = q_decode(C, D, H, RB, RPW, ny, TZ, nz, WQ);
  const long long cofs = (long long)b.c * D * HW;
  const float* dzp = dz + (long long)b.n * dzns + cofs;
  const T* xp = x + (long long)b.n * xns + cofs;
  float sc = 1.f, sh = 0.f, mu = 0.f;
  if (XF) {
    const float* r = rec + (long long)b.nc * kRec;
    mu = r[0]; sc = r[2]; sh = r[3];
  }
  for (int i = threadIdx.x; i < 2 * PP; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f4 g0 = zero4, g1 = zero4, g2 = zero4;   // own dZ of planes za-1, za, za+1
  f2 gw[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) gw[t] = f2{0.f, 0.f};
  const int zlo = max(0, b.z0 - 1), zhi = min(D - 1, b.z1);
  const QMap qm = q_map(b.y0, b.rows, H, W, WQ);
  auto zc = [&](int z) { return (long long)min(max(z, zlo), zhi) * HW; };
  const long long qofs = (long long)(b.y0 + b.oy) * W + b.ox;
  auto dzq = [&](int z) {   // own dZ quad of plane z (clamped address, always issued)
    return ldv4(dzp + (long long)min(max(z, 0), D - 1) * HW + qofs);
  };
  QPre<T> p0, p1;
  q_fetch(p0, xp + zc(b.z0 - 1), qm);
  q_fetch(p1, xp + zc(b.z0), qm);
  f4 q0 = dzq(b.z0), q1 = dzq(b.z0 + 1);
  auto step = [&](int t, QPre<T>& pre, f4& q) {
    const int za = b.z0 - 1 + t;   // A plane of this step
    float* buf = lds + (t & 1) * PP;
    q_commit<XF == 1>(pre, buf, qm, za >= zlo && za <= zhi, sc, mu, sh);
    q_fetch(pre, xp + zc(za + 2), qm);
    g0 = g1;
    g1 = g2;
    const int zd = za + 1;
    g2 = (b.own && zd >= b.z0 && zd < b.z1) ? q : zero4;
    q = dzq(zd + 2);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float u[6];
      q_nbr(buf, b.oy + r, W, b.ox, b.el, b.er, u);
#pragma unroll
      for (int dxi = 0; dxi < 3; ++dxi) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {   // x-pairs (2h, 2h+1): one v_pk_fma_f32 per tap and kd
          const f2 uu = {u[2 * h + dxi], u[2 * h + 1 + dxi]};
          gw[r * 3 + dxi] = pfma(f2{g2[2 * h], g2[2 * h + 1]}, uu, gw[r * 3 + dxi]);            // kd=0
          gw[9 + r * 3 + dxi] = pfma(f2{g1[2 * h], g1[2 * h + 1]}, uu, gw[9 + r * 3 + dxi]);    // kd=1
          gw[18 + r * 3 + dxi] = pfma(f2{g0[2 * h], g0[2 * h + 1]}, uu, gw[18 + r * 3 + dxi]);  // kd=2
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 27; ++k) pin(gw[k]);
  };
#pragma unroll
  for (int t = 0; t < TZC + 2; t += 2) {
    step(t, p0, q0);
    step(t + 1, p1, q1);
  }
  __syncthreads();
  float* red = lds;   // [nwaves][32]
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    const float r = wave_sum(gw[t].x + gw[t].y);
    if (ln == 0) red[wv * 32 + t] = r;
  }
  __syncthreads();
  const int nchunk = nz * ny;
  if (threadIdx.x < 27) {
    float r = 0.f;
    for (int k = 0; k < nw; ++k) r += red[k * 32 + threadIdx.x];
    dw_part[((long long)b.c * N * nchunk + (long long)b.n * nchunk + b.ck) * 27 + threadIdx.x] = r;
  }
}

// ------------------------------------------------------------------------------------------------
// Single-pass backward with packed FP32 FMAs (v_pk_fma_f32): data gradient AND weight gradient
// from one read of dZ and A and one write of dX (3 tensors of HBM traffic instead of the split
// passes' 4).  The 54 FMAs per voxel are what bounded the earlier fused kernel (VALU-bound at one
// FMA per instruction); here almost all of them issue two per instruction:
//   data   dA(plane p)[i] += wf(kd, r, dx) * dZ(zd, row r)[i + dx]   (wf = flipped taps)
//          planes zd-1 (kd 0) and zd (kd 1) are one accumulator PAIR per voxel i, multiplied by
//          the tap PAIR (wf(0,.), wf(1,.)) (uniform: SGPRs) and the neighbour broadcast through
//          op_sel; plane zd+1 (kd 2) pairs voxels (i, i+1) where the neighbour pair is an
//          aligned register pair (dx = 1), scalar otherwise.
//   weight gw(kd, r, dx) += sum_i g_kd[i] * A(za, row r)[i + dx]   (g_kd = own dZ quad of
//          plane za+1-kd): per (kd, r) the pairs (dx 0, dx 1) and (dx 1, dx 2) take the voxels
//          whose neighbour pair is aligned (i = 1, 3 and i = 0, 2), four products stay scalar.
// The step index is a compile-time constant (index_sequence expansion), so the boundary steps
// skip the work that only touches planes outside the slab: per owned voxel the kernel issues
// exactly the 27 + 27 tap products.
// ------------------------------------------------------------------------------------------------
// the single-pass backward: occupancy target and register prefetch depth of the register-staged
// form; the LDS-DMA form's DMA ring depth and occupancy (the IN-fused MODE 1: 3 waves, 4 spill)
#ifndef L3U_DWG_PD
#define L3U_DWG_PD 1
#endif
constexpr int kDwpWaves = 3, kDwpPd = 2;
constexpr int kDwgPd = L3U_DWG_PD, kDwgWaves = 4, kDwgWaves1 = 3;

template <class F, int... I>
L3U_DEV void run_steps(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// LDS row image of the packed kernel: unpadded rows (pitch W), one ds_read_b128 per row quad, the
// x-neighbours by DPP from the adjacent lanes (measured faster than a padded image read with
// ds_read_b64 neighbour pairs: ds_read2_b64 costs 8 LDS cycles vs 4 for b128, and the LDS pipe
// also carries the ds_write_b128 commits at ~13 cycles each)
constexpr int kLPad = 0, kLOfs = 0;
constexpr int kNH = 0;   // half of n2 holding x-1

// row read: n2[kNH] = x-1, m = x..x+3, p2.x = x+4 (zero beyond the row)
L3U_DEV void q_row3(const float* plane, int row, int lp, int ox, bool el, bool er, f2& n2, f4& m,
                    f2& p2) {
  const float* q = plane + row * lp + ox;
  m = *reinterpret_cast<const f4*>(q);
  const float pl = lane_prev(m[3]), pr = lane_next(m[0]);
  const float l = el ? 0.f : pl, r = er ? 0.f : pr;
  n2 = f2{l, l};
  p2 = f2{r, r};
}

// the same from an already-read quad m0 (neighbours by DPP, or from LDS in the padded layout)
template <typename LT>
L3U_DEV void q_nbr3(const f4& m0, const LT* plane, int row, int lp, int ox, bool el, bool er,
                    f2& n2, f4& m, f2& p2) {
  m = m0;
  const float pl = lane_prev(m[3]), pr = lane_next(m[0]);
  const float l = el ? 0.f : pl, r = er ? 0.f : pr;
  n2 = f2{l, l};
  p2 = f2{r, r};
}

// acc + a * {b[H], b[H]}: the product with one half of an aligned register pair broadcast to both
// lanes of the packed FMA (op_sel picks the half; the compiler only folds the low-half case)
template <int H>
L3U_DEV f2 pk_bc(f2 acc, f2 a, f2 b) {
  if (H == 0) return pfma(a, f2{b.x, b.x}, acc);
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}
// scalar FMAs kept scalar: left to the SLP vectorizer, neighbouring ones get packed with v_mov
// pairing that costs more than it saves
L3U_DEV float sfma_s(float acc, float a, float b) {   // a wave-uniform
  asm("v_fmac_f32 %0, %1, %2" : "+v"(acc) : "s"(a), "v"(b));
  return acc;
}
L3U_DEV float sfma_v(float acc, float a, float b) {
  asm("v_fmac_f32 %0, %1, %2" : "+v"(acc) : "v"(a), "v"(b));
  return acc;
}
template <int H>
L3U_DEV f2 pk_bc_s(f2 acc, f2 a, f2 b) {   // a wave-uniform (SGPR pair)
  if (H == 0) return pfma(a, f2{b.x, b.x}, acc);
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(a), "v"(b));
  return acc;
}

// LDS-DMA staging (GL = true, one-wave tiles): each plane goes global -> LDS with
// global_load_lds_dwordx4 (no staging VGPRs, no ds_write), PD planes ahead in a ring of PD + 1
// buffers of 128 quads per tensor.  Lane l of slot k lands at quad 64k + l, which is the q_map
// order; lanes whose quad lies outside the volume (rows y = -1 / H, planes z = -1 / D) or past
// the tile (slot-1 tail) read a zero page instead, so every wave issues exactly 2 DMAs per
// tensor per step and the waits are static counts.  The DMA is inline asm (M0 is written in the
// same statement), so its completion is counted here, not by the compiler: see dw_wait_vm.
__device__ __attribute__((aligned(16))) float g_l3u_zero_page[256];   // 1 KiB of zeros (64 lanes x 16 B)

L3U_DEV void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// DMAs issued for plane step t (slots per loaded tensor: 2 for fp32, 1 for bf16 — NSD for dZ,
// NSA for A; see gissue)
template <int TZC, int NSD, int NSA>
constexpr int gl_n(int t) { return NSD * (t < TZC + 2 ? 1 : 0) + NSA * (t > 0 ? 1 : 0); }
// DMAs younger than plane step s's when step s waits for it (planes s+1 .. s+PD, if issued)
template <int TZC, int PD, int NSD, int NSA>
constexpr int gl_younger(int s) {
  int n = 0;
  for (int t = s + 1; t <= s + PD && t < TZC + 3; ++t) n += gl_n<TZC, NSD, NSA>(t);
  return n;
}
template <int NOUT>
L3U_DEV void dw_wait_vm() {   // at most NOUT vector-memory operations still outstanding
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NOUT) : "memory");
}

// Gradients (dZ, dX) are fp32; the saved activation A is T (fp32, or bf16 in the bf16 network).
// bf16 A on the LDS-DMA path: the DMA moves raw bf16, 8 elements (two quads) per lane, so one
// slot per plane covers the 128-quad tile (needs an even quad count per row, W % 8 == 0, so a
// lane's pair never straddles a row); that LDS image is bf16 and its rows widen at the read.
template <typename T, int MODE, int TZC, bool GL = false, bool XR1 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GL ? (MODE == 1 ? kDwgWaves1 : kDwgWaves) : kDwpWaves))) void dw3p_bwd_kernel(
    const float* __restrict__ dz, long long dzns, const T* __restrict__ x, long long xns,
    const float* __restrict__ w, const float* __restrict__ rec, float* __restrict__ dx,
    long long dxns, float* __restrict__ dw_part, double* __restrict__ in_part,
    int N, int C, int D, int H, int W, int RB, int RPW, int ny, int TZ, int nz) {
  L3U_STAMP_SCOPE(205);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using LTA = std::conditional_t<GL, T, float>;        // LDS element type of the A image
  constexpr bool BH = GL && sizeof(T) == 2;
  constexpr int NSA = BH ? 1 : 2;                      // DMA slots per A plane (dZ: 2)
  const int WQ = W >> 2, LP = W + kLPad, PP = (RB + 2) * LP, HW = H * W;
  const QBlock b = q_decode(C, D, H, RB, RPW, ny, TZ, nz, WQ);
  const long long cofs = (long long)b.c * D * HW;
  // XR1 (xns < 0, GL + MODE 1): a rank-1 input, channel c = rec[c][7] * one stored channel
  // (include/l3u.h); a template flag so that the other variants keep their schedule
  constexpr bool xk = GL && MODE == 1 && XR1;
  const float* dzp = dz + (long long)b.n * dzns + cofs;
  const T* xp = x + (long long)b.n * (xk ? -xns : xns) + (xk ? 0ll : cofs);
  float* dxp = dx + (long long)b.n * dxns + cofs;
  constexpr int GNB = kDwgPd + 1;                  // DMA ring buffers per tensor
  const int GPSD = (RB + 2) * W;                       // dZ elements per ring buffer (nq quads)
  const int GPSA = BH ? 512 : (RB + 2) * W;            // A elements per ring buffer
  float* const dzl = lds;                              // dZ planes
  LTA* const al = reinterpret_cast<LTA*>(lds + (GL ? GNB * GPSD : 2 * PP));   // A planes
  // flipped data-gradient taps: pair (kd 0, kd 1) and kd 2 per in-plane tap (r, dx)
  f2 wp[9];
  float w2[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int tf = 8 - t;
    wp[t] = f2{w[b.c * 27 + tf], w[b.c * 27 + 9 + tf]};
    w2[t] = w[b.c * 27 + 18 + tf];
  }
  float sc = 1.f, sh = 0.f, kk = 1.f, mean = 0.f, rstd = 1.f, rks = 1.f;
  if (MODE == 1) {
    const float* r = rec + (long long)b.nc * kRec;
    mean = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4]; rks = r[7];
  }
  if (!GL)
    for (int i = threadIdx.x; i < 4 * PP; i += blockDim.x) lds[i] = 0.f;
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const f2 zero2 = {0.f, 0.f};
  f2 P[4];                      // (dA plane zd-1, dA plane zd) per voxel of the quad
  f2 S01 = zero2, S23 = zero2;  // dA plane zd+1, voxels (0,1), (2,3)
#pragma unroll
  for (int i = 0; i < 4; ++i) P[i] = zero2;
  f2 GA[9], GB[9];              // per (kd, r): (gw dx0, gw dx1 part a), (gw dx1 part b, gw dx2)
#pragma unroll
  for (int t = 0; t < 9; ++t) GA[t] = GB[t] = zero2;
  f4 g0 = zero4, g1 = zero4, g2 = zero4;   // own dZ quads of planes zd, zd-1, zd-2
  float s1 = 0.f, s2 = 0.f;
  const int zlo = max(0, b.z0 - 1), zhi = min(D - 1, b.z1);
  const long long qofs = (long long)(b.y0 + b.oy) * W + b.ox;
  // register staging PD planes ahead (sets alternate by step parity when PD = 2)
  constexpr int PD = GL ? 1 : kDwpPd;
  QPre<float> pzs[PD];
  QPre<T> pas[PD];
  const QMap qm = q_map(b.y0, b.rows, H, W, WQ, LP, kLOfs);
  auto in_rng = [&](int z) { return z >= zlo && z <= zhi; };
  auto zc = [&](int z) { return (long long)min(max(z, zlo), zhi) * HW; };
  const unsigned lbase = (unsigned)(size_t)lds;
  float rv[3];   // MODE 1 (GL): row r of the thread's 3-row window lies inside the volume
#pragma unroll
  for (int r = 0; r < 3; ++r) rv[r] = (unsigned)(b.y0 + b.oy + r - 1) < (unsigned)H ? 1.f : 0.f;
  const float* zpage = g_l3u_zero_page + 4 * (threadIdx.x & 63);
  // bf16: lane l moves quads 2l, 2l+1 of the tile (same row: W % 8 == 0)
  int goff2 = 0;
  bool ok2 = false;
  if (BH) {
    const int qp = 2 * (int)(threadIdx.x & 63), lr2 = qp / WQ, y2 = b.y0 - 1 + lr2;
    ok2 = qp < (RB + 2) * WQ && y2 >= 0 && y2 < H;
    goff2 = min(max(y2, 0), H - 1) * W + (qp - lr2 * WQ) * 4;
  }
  // DMA of plane step t (dZ plane z0-1+t, A plane z0-2+t) into ring buffer t % GNB.  Step 0's A
  // plane and the last step's dZ plane are never used: not loaded (gl_n gives the DMA count).
  // Slot 1 is issued by the lanes of its nq - 64 quads only (nq > 64 for one-wave tiles, so the
  // instruction always issues and the count stays static).
  const int nq = (RB + 2) * WQ;
  auto gissue = [&](auto TI) {
    constexpr int t = decltype(TI)::value;
    const int z_d = b.z0 - 1 + t, z_a = z_d - 1;
    const bool ind = in_rng(z_d), ina = in_rng(z_a);
    const unsigned bz = lbase + (unsigned)((t % GNB) * GPSD) * 4u;
    const unsigned ba = (unsigned)(size_t)al + (unsigned)((t % GNB) * GPSA) * (unsigned)sizeof(T);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && (int)threadIdx.x >= nq - 64) continue;
      const void* sd = (qm.ok[k] && ind) ? (const void*)(dzp + (long long)z_d * HW + qm.goff[k]) : (const void*)zpage;
      if constexpr (t < TZC + 2) glds16(sd, bz + k * 1024u);
      if constexpr (!BH) {
        const void* sa = (qm.ok[k] && ina) ? (const void*)(xp + (long long)z_a * HW + qm.goff[k]) : (const void*)zpage;
        if constexpr (t > 0) glds16(sa, ba + k * 1024u);
      }
    }
    if constexpr (BH) {
      const void* sa = (ok2 && ina) ? (const void*)(xp + (long long)z_a * HW + goff2) : (const void*)zpage;
      if constexpr (t > 0) glds16(sa, ba);
    }
  };
  if constexpr (GL) {
    run_steps(gissue, std::make_integer_sequence<int, kDwgPd>{});
  } else {
#pragma unroll
    for (int k = 0; k < PD; ++k) {
      q_fetch(pzs[k], dzp + zc(b.z0 - 1 + k), qm);
      q_fetch(pas[k], xp + zc(b.z0 - 2 + k), qm);
    }
  }
  __syncthreads();
  auto step = [&](auto I) {
    constexpr int s = decltype(I)::value;
    QPre<float>& pz = pzs[s % PD];
    QPre<T>& pa = pas[s % PD];
    // planes of the slab are z0 .. z0+TZC-1 (z1 may cut it short at run time)
    constexpr bool doP = s >= 1 && s <= TZC + 1;    // dA planes zd-1 / zd touch the slab
    constexpr bool doS = s <= TZC - 1;              // dA plane zd+1 in the slab
    constexpr bool own0 = s >= 1 && s <= TZC;       // dZ plane zd owned
    constexpr bool use1 = s >= 2 && s <= TZC + 1;   // dZ plane zd-1 owned
    constexpr bool use2 = s >= 3 && s <= TZC + 2;   // dZ plane zd-2 owned
    constexpr bool fin = s >= 2 && s <= TZC + 1;    // dA plane zd-1 completes in the slab
    const int zd = b.z0 - 1 + s, za = zd - 1;
    float* dbuf = GL ? dzl + (s % GNB) * GPSD : dzl + (s & 1) * PP;
    LTA* abuf = GL ? al + (s % GNB) * GPSA : al + (s & 1) * PP;
    if constexpr (GL) {
      // issue plane s + PD (its ring buffer was last read in step s - 1), then wait for plane s:
      // younger than plane s's 4 DMAs are those of planes s+1 .. s+PD (stores between them only
      // make the wait longer)
      if constexpr (s + kDwgPd < TZC + 3) gissue(std::integral_constant<int, s + kDwgPd>{});
      dw_wait_vm<gl_younger<TZC, kDwgPd, 2, NSA>(s)>();
    } else {
      q_commit<false>(pz, dbuf, qm, in_rng(zd), 1.f, 0.f, 0.f);
      q_commit<MODE == 1>(pa, (float*)abuf, qm, in_rng(za), sc, mean, sh);
      if constexpr (s + PD < TZC + 3) {
        q_fetch(pz, dzp + zc(zd + PD), qm);
        q_fetch(pa, xp + zc(za + PD), qm);
      }
    }
    const int zf = zd - 1;
    f4 epi = zero4;
    // GL + MODE 1: the pre-IN activation of plane zf = za is the tile's own raw A row in LDS
    if constexpr (MODE == 1 && fin && !GL)
      epi = ldv4(xp + (long long)min(max(zf, 0), D - 1) * HW + qofs);
    if constexpr (MODE == 2 && fin)
      epi = ldv4(dxp + (long long)min(max(zf, 0), D - 1) * HW + qofs);
    __syncthreads();
    // all six LDS rows of the step are read up front (one latency for the step, not three)
    constexpr bool needD = doP || doS || own0, needA = own0 || use1 || use2;
    f4 rowd[3], rowa[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      if (needD) rowd[r] = ldv4(dbuf + (b.oy + r) * LP + kLOfs + b.ox);
      if (needA) rowa[r] = ldv4(abuf + (b.oy + r) * LP + kLOfs + b.ox);
    }
    f4 pre1 = zero4, d1 = zero4;   // GL + MODE 1: own row's pre-activation and (y - mean)
    if constexpr (GL && MODE == 1 && needA) {
      // the DMA staged y itself: A = lrelu(scale*(y-mean)+shift) is formed at the read (packed
      // ops), with the conv's zero padding in the A domain: rows / planes outside the volume
      // hold zero-page values and get scale = shift = 0
      float zm = in_rng(za) ? 1.f : 0.f;
      pin(zm);   // formed here: keeps the compiler from hoisting 3 x (TZC+3) masks
      if (xk) {   // rank-1 input: the channel's value, the materialised product bit for bit
#pragma unroll
        for (int r = 0; r < 3; ++r) rowa[r] = mul_rn(rowa[r], rks);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const float mr = zm * rv[r];
        const f2 sc2 = {sc * mr, sc * mr}, sh2 = {sh * mr, sh * mr}, mu2 = {mean, mean};
        f2 lo = f2{rowa[r][0], rowa[r][1]} - mu2, hi = f2{rowa[r][2], rowa[r][3]} - mu2;
        if (fin && r == 1) d1 = f4{lo.x, lo.y, hi.x, hi.y};
        lo = pfma(sc2, lo, sh2);
        hi = pfma(sc2, hi, sh2);
        if (fin && r == 1) pre1 = f4{lo.x, lo.y, hi.x, hi.y};
        const f2 ls = lo * f2{kSlope, kSlope}, hs = hi * f2{kSlope, kSlope};
        rowa[r] = f4{fmaxf(lo.x, ls.x), fmaxf(lo.y, ls.y), fmaxf(hi.x, hs.x), fmaxf(hi.y, hs.y)};
      }
    }
    if constexpr (needD) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        f2 n2, p2;
        f4 m;
        q_nbr3(rowd[r], dbuf, b.oy + r, LP, b.ox, b.el, b.er, n2, m, p2);
        const f2 m01 = {m[0], m[1]}, m23 = {m[2], m[3]};
        if (r == 1 && own0) g0 = (b.own && zd < b.z1) ? m : zero4;
        if constexpr (doP) {
          // v[j] = x-1+j: l = n2.hi, m0 = m01.lo, m1 = m01.hi, m2 = m23.lo, m3 = m23.hi, r = p2.lo
          const f2 w0 = wp[r * 3], w1 = wp[r * 3 + 1], w2p = wp[r * 3 + 2];
          P[0] = pk_bc_s<kNH>(P[0], w0, n2);  P[0] = pk_bc_s<0>(P[0], w1, m01); P[0] = pk_bc_s<1>(P[0], w2p, m01);
          P[1] = pk_bc_s<0>(P[1], w0, m01); P[1] = pk_bc_s<1>(P[1], w1, m01); P[1] = pk_bc_s<0>(P[1], w2p, m23);
          P[2] = pk_bc_s<1>(P[2], w0, m01); P[2] = pk_bc_s<0>(P[2], w1, m23); P[2] = pk_bc_s<1>(P[2], w2p, m23);
          P[3] = pk_bc_s<0>(P[3], w0, m23); P[3] = pk_bc_s<1>(P[3], w1, m23); P[3] = pk_bc_s<0>(P[3], w2p, p2);
        }
        if constexpr (doS) {
          const float a0 = w2[r * 3], a1 = w2[r * 3 + 1], a2 = w2[r * 3 + 2];
          S01.x = sfma_s(S01.x, a0, n2.y);
          S01.y = sfma_s(S01.y, a0, m[0]);
          S23.x = sfma_s(S23.x, a0, m[1]);
          S23.y = sfma_s(S23.y, a0, m[2]);
          S01 = pfma(f2{a1, a1}, m01, S01);
          S23 = pfma(f2{a1, a1}, m23, S23);
          S01.x = sfma_s(S01.x, a2, m[1]);
          S01.y = sfma_s(S01.y, a2, m[2]);
          S23.x = sfma_s(S23.x, a2, m[3]);
          S23.y = sfma_s(S23.y, a2, p2.x);
        }
      }
    }
    if constexpr (needA) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        f2 n2, p2;
        f4 m;
        q_nbr3(rowa[r], abuf, b.oy + r, LP, b.ox, b.el, b.er, n2, m, p2);
        const f2 m01 = {m[0], m[1]}, m23 = {m[2], m[3]};
        auto acc = [&](const f4& g, f2& A, f2& B) {
          const f2 g01 = {g[0], g[1]}, g23 = {g[2], g[3]};
          A = pk_bc<1>(A, m01, g01);   // g1 * (m0, m1)
          A = pk_bc<1>(A, m23, g23);   // g3 * (m2, m3)
          B = pk_bc<0>(B, m01, g01);   // g0 * (m0, m1)
          B = pk_bc<0>(B, m23, g23);   // g2 * (m2, m3)
          A.x = sfma_v(A.x, g[0], n2.y);
          A.x = sfma_v(A.x, g[2], m[1]);
          B.y = sfma_v(B.y, g[1], m[2]);
          B.y = sfma_v(B.y, g[3], p2.x);
        };
        if constexpr (own0) acc(g0, GA[r], GB[r]);          // kd 0: dZ plane za+1 = zd
        if constexpr (use1) acc(g1, GA[3 + r], GB[3 + r]);  // kd 1: dZ plane za = zd-1
        if constexpr (use2) acc(g2, GA[6 + r], GB[6 + r]);  // kd 2: dZ plane za-1 = zd-2
      }
    }
    if constexpr (fin) {
      f4 o = {P[0].x, P[1].x, P[2].x, P[3].x};
      const bool st = b.own && zf < b.z1;
      if (MODE == 1 && GL) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dp = o[i] * kk * lrelu_d(pre1[i]);
          o[i] = dp;
          s1 += st ? dp : 0.f;
          s2 += st ? dp * (d1[i] * rstd) : 0.f;
        }
      } else if (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pre = fmaf(sc, epi[i] - mean, sh);
          const float dp = o[i] * kk * lrelu_d(pre);
          o[i] = dp;
          s1 += st ? dp : 0.f;
          s2 += st ? dp * ((epi[i] - mean) * rstd) : 0.f;
        }
      } else if (MODE == 2) {
        o += epi;
      }
      if (st) {
        float* dst = dxp + (long long)zf * HW + qofs;
        if (GL) stv4_nt(dst, o);   // streamed out, not re-read (non-temporal: -0.8 us at [4,32,48^3])
        else stv4(dst, o);
      }
    }
    // keep each step's accumulation inside the step (no sinking of FMAs past later barriers)
#pragma unroll
    for (int t = 0; t < 9; ++t) { pin(GA[t]); pin(GB[t]); }
#pragma unroll
    for (int i = 0; i < 4; ++i) pin(P[i]);
    pin(S01);
    pin(S23);
    if constexpr (MODE == 1 && fin) { pin(s1); pin(s2); }   // else the IN sums sink to the end
    P[0] = f2{P[0].y, S01.x};
    P[1] = f2{P[1].y, S01.y};
    P[2] = f2{P[2].y, S23.x};
    P[3] = f2{P[3].y, S23.y};
    S01 = S23 = zero2;
    g2 = g1;
    g1 = g0;
  };
  run_steps(step, std::make_integer_sequence<int, TZC + 3>{});
  // fixed-order workgroup reduction of the 27 taps (+ the IN sums)
  __syncthreads();
  float* red = lds;                                        // [nwaves][32]
  double* redd = reinterpret_cast<double*>(lds + 4 * 32);  // [nwaves][2]
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int t = 0; t < 9; ++t) {   // t = kd * 3 + r
    const float r0 = wave_sum(GA[t].x), r1 = wave_sum(GA[t].y + GB[t].x), r2 = wave_sum(GB[t].y);
    if (ln == 0) {
      red[wv * 32 + t * 3 + 0] = r0;
      red[wv * 32 + t * 3 + 1] = r1;
      red[wv * 32 + t * 3 + 2] = r2;
    }
  }
  if (MODE == 1) {
    const double r1 = wave_sum_d((double)s1), r2 = wave_sum_d((double)s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
  }
  __syncthreads();
  const int nchunk = nz * ny;
  if (threadIdx.x < 27) {
    float r = 0.f;
    for (int k = 0; k < nw; ++k) r += red[k * 32 + threadIdx.x];
    dw_part[((long long)b.c * N * nchunk + (long long)b.n * nchunk + b.ck) * 27 + threadIdx.x] = r;
  }
  if (MODE == 1 && threadIdx.x >= 32 && threadIdx.x < 34) {
    const int j = threadIdx.x - 32;
    double r = 0.0;
    for (int k = 0; k < nw; ++k) r += redd[k * 2 + j];
    in_part[(((long long)b.c * N + b.n) * nchunk + b.ck) * 2 + j] = r;
  }
}

// ------------------------------------------------------------------------------------------------
// Forward stencil on the single pass's machinery (l3u_dw3_fwd, planes >= 12^2, one-wave tiles):
// the input planes go global -> LDS by LDS-DMA, a ring of PD + 1 plane buffers (no staging VGPRs,
// a deeper prefetch than dw3q_fwd's two register-staged planes), and the 27 tap products per voxel
// issue mostly as v_pk_fma_f32: output planes (zi-1, zi) of a voxel are one accumulator PAIR,
// multiplied by the tap pair (kd 2, kd 1) from SGPRs with the neighbour broadcast by op_sel, and
// plane zi+1 (kd 0) pairs voxels (i, i+1) where the neighbour pair is register-aligned -- the data
// path of dw3p_bwd_kernel with unflipped taps (24 + 12 packed and 12 scalar FMAs per row quad and
// input plane, against dw3q_fwd's 36 scalar ones).
//   XF = 1: the input is transformed on load, a = lrelu(scale*(x-mean)+shift) (IN1 + LeakyReLU +
//           Dropout3d before conv2.depthwise), applied to the rows read from LDS with packed ops;
//           rows / planes outside the volume get scale = shift = 0 so the zero page stays a zero
//           in the A domain; the record is finalized in-kernel when has_src.
// The output quad is written through a buffer descriptor with an out-of-range offset for lanes
// that own no voxel, so every wave issues exactly one store per output plane and the DMA waits
// are exact compile-time counts that include the stores.
// ------------------------------------------------------------------------------------------------
#ifndef L3U_DWF_PD
#define L3U_DWF_PD 2
#endif
constexpr int kDwfPd = L3U_DWF_PD;   // planes in flight ahead of the one being consumed
#ifndef L3U_DWF_GL
#define L3U_DWF_GL 1
#endif
constexpr bool kDwfGl = L3U_DWF_GL != 0;   // the forward on dw3g_fwd_kernel (0: dw3q_fwd)
#ifndef L3U_DWF_AUX
#define L3U_DWF_AUX 2
#endif
// cache bits of the output stores: 2 = nt (r5 A/B vs 0: -2..-3.5 us/step; 16 = sc1
// write-through -1..-2 us)
constexpr int kDwfAux = L3U_DWF_AUX;

template <int TZC, int NS, int PD>
constexpr int gf_younger(int s) {   // vm ops younger than plane s's DMAs when step s waits
  int n = 0;
  for (int t = s + 1; t <= s + PD && t < TZC + 2; ++t) n += NS;   // DMAs of planes s+1 .. s+PD
  // stores of steps s-PD .. s-1 (issued after plane s's DMAs, which went out at step s-PD)
  for (int t = s - PD; t < s; ++t) n += (t >= 2 && t <= TZC + 1) ? 1 : 0;
  return n;
}

template <typename T, int XF, int TZC, bool XR1 = false>
__global__ __launch_bounds__(64) void dw3g_fwd_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    const float* __restrict__ rec, l3u_norm_src src, int has_src, T* __restrict__ y,
    long long yns, int N, int C, int D, int H, int W, int RB, int RPW, int ny, int TZ, int nz) {
  L3U_STAMP_SCOPE(209);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr bool BH = sizeof(T) == 2;
  constexpr int NS = BH ? 1 : 2;          // DMA slots per plane
  constexpr int PD = kDwfPd, GNB = PD + 1;
  using LT = T;                           // LDS element type of the plane image
  const int WQ = W >> 2, HW = H * W;
  const QBlock b = q_decode(C, D, H, RB, RPW, ny, TZ, nz, WQ);
  const long long cofs = (long long)b.c * D * HW;
  // XR1 (xns < 0, XF, fp32): a rank-1 input, channel c = rec[c][7] * one stored channel
  // (include/l3u.h "Rank-1 operands"): the first block's y1 = w1[c] * z1, never materialised
  const T* xp = x + (long long)b.n * (XR1 ? -xns : xns) + (XR1 ? 0ll : cofs);
  T* yp = y + (long long)b.n * yns + cofs;
  const int GPS = BH ? 512 : (RB + 2) * W;   // elements per ring buffer
  LT* const ring = reinterpret_cast<LT*>(lds);
  const int zlo = max(0, b.z0 - 1), zhi = min(D - 1, b.z1);
  auto in_rng = [&](int z) { return z >= zlo && z <= zhi; };
  const QMap qm = q_map(b.y0, b.rows, H, W, WQ);
  const float* zpage = g_l3u_zero_page + 4 * (threadIdx.x & 63);
  int goff2 = 0;
  bool ok2 = false;
  if (BH) {   // lane l moves quads 2l, 2l+1 (one row: W % 8 == 0)
    const int qp = 2 * (int)threadIdx.x, lr2 = qp / WQ, y2 = b.y0 - 1 + lr2;
    ok2 = qp < (RB + 2) * WQ && y2 >= 0 && y2 < H;
    goff2 = min(max(y2, 0), H - 1) * W + (qp - lr2 * WQ) * 4;
  }
  const int nq = (RB + 2) * WQ;
  const unsigned lbase = (unsigned)(size_t)lds;
  auto gissue = [&](auto TI) {   // input plane z0-1+t -> ring buffer t % GNB
    constexpr int t = decltype(TI)::value;
    const int zi = b.z0 - 1 + t;
    const bool in = in_rng(zi);
    const unsigned bz = lbase + (unsigned)((t % GNB) * GPS) * (unsigned)sizeof(T);
    if constexpr (BH) {
      const void* s = (ok2 && in) ? (const void*)(xp + (long long)zi * HW + goff2) : (const void*)zpage;
      glds16(s, bz);
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k == 1 && (int)threadIdx.x >= nq - 64) continue;
        const void* s = (qm.ok[k] && in) ? (const void*)(xp + (long long)zi * HW + qm.goff[k]) : (const void*)zpage;
        glds16(s, bz + k * 1024u);
      }
    }
  };
  RecPre rp;
  if (XF && has_src) record_pre(src, b.n, b.c, C, rp);   // the partials, beside the first DMAs
  run_steps(gissue, std::make_integer_sequence<int, PD>{});
  // taps: pair (kd 2, kd 1) and kd 0 per in-plane tap t = r * 3 + dx
  f2 wp[9];
  float w0[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wp[t] = f2{w[b.c * 27 + 18 + t], w[b.c * 27 + 9 + t]};
    w0[t] = w[b.c * 27 + t];
  }
  float sc = 1.f, sh = 0.f, mu = 0.f, rks = 1.f;
  if (XF) {
    if (has_src) {   // one-wave tiles: the wave merges the record itself
      float r8[kRec];
      record_finish(src, rp, b.n, b.c, C, r8);
      mu = r8[0]; sc = r8[2]; sh = r8[3]; rks = r8[7];
      if (b.ck == 0 && threadIdx.x == 0 && src.rec_out) {
        float* o = src.rec_out + (long long)b.nc * kRec;
#pragma unroll
        for (int i = 0; i < kRec; ++i) o[i] = r8[i];
      }
    } else {
      const float* r = rec + (long long)b.nc * kRec;
      mu = r[0]; sc = r[2]; sh = r[3]; rks = r[7];
    }
  }
  float rv[3];   // XF: row r of the thread's 3-row window lies inside the volume
#pragma unroll
  for (int r = 0; r < 3; ++r) rv[r] = (unsigned)(b.y0 + b.oy + r - 1) < (unsigned)H ? 1.f : 0.f;
  // the output store: quad (oy, ox) of plane zf; lanes owning no voxel get an offset past the
  // descriptor's range (the store is dropped), so the store always issues
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      yp, 0, (int)min((long long)D * HW * (long long)sizeof(T), 0x7fffffffll), 0x00020000);
  const unsigned qoff = b.own ? (unsigned)(((b.y0 + b.oy) * W + b.ox) * (int)sizeof(T)) : 0x80000000u;
  const f2 zero2 = {0.f, 0.f};
  f2 P[4];                      // (plane zi-1, plane zi) per voxel of the quad
  f2 S01 = zero2, S23 = zero2;  // plane zi+1, voxels (0,1), (2,3)
#pragma unroll
  for (int i = 0; i < 4; ++i) P[i] = zero2;
  auto step = [&](auto I) {
    constexpr int s = decltype(I)::value;
    constexpr bool doP = s >= 1 && s <= TZC + 1;
    constexpr bool doS = s <= TZC - 1;
    constexpr bool fin = s >= 2 && s <= TZC + 1;
    const int zi = b.z0 - 1 + s;
    const LT* buf = ring + (s % GNB) * GPS;
    // issue plane s + PD (its buffer was last read in step s - 1, behind that step's barrier),
    // then wait for plane s
    if constexpr (s + PD < TZC + 2) gissue(std::integral_constant<int, s + PD>{});
    dw_wait_vm<gf_younger<TZC, NS, PD>(s)>();
    __syncthreads();
    if constexpr (doP || doS) {
      f4 row[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) row[r] = ldv4(buf + (b.oy + r) * W + b.ox);
      if constexpr (XF == 1) {
        float zm = in_rng(zi) ? 1.f : 0.f;
        pin(zm);
        if constexpr (XR1) {   // the channel's value: the materialised product, bit for bit
#pragma unroll
          for (int r = 0; r < 3; ++r) row[r] = mul_rn(row[r], rks);
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const float mr = zm * rv[r];
          const f2 sc2 = {sc * mr, sc * mr}, sh2 = {sh * mr, sh * mr}, mu2 = {mu, mu};
          f2 lo = f2{row[r][0], row[r][1]} - mu2, hi = f2{row[r][2], row[r][3]} - mu2;
          lo = pfma(sc2, lo, sh2);
          hi = pfma(sc2, hi, sh2);
          const f2 ls = lo * f2{kSlope, kSlope}, hs = hi * f2{kSlope, kSlope};
          row[r] = f4{fmaxf(lo.x, ls.x), fmaxf(lo.y, ls.y), fmaxf(hi.x, hs.x), fmaxf(hi.y, hs.y)};
        }
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        f2 n2, p2;
        f4 m;
        q_nbr3(row[r], buf, b.oy + r, W, b.ox, b.el, b.er, n2, m, p2);
        const f2 m01 = {m[0], m[1]}, m23 = {m[2], m[3]};
        if constexpr (doP) {
          const f2 t0 = wp[r * 3], t1 = wp[r * 3 + 1], t2 = wp[r * 3 + 2];
          P[0] = pk_bc_s<kNH>(P[0], t0, n2); P[0] = pk_bc_s<0>(P[0], t1, m01); P[0] = pk_bc_s<1>(P[0], t2, m01);
          P[1] = pk_bc_s<0>(P[1], t0, m01);  P[1] = pk_bc_s<1>(P[1], t1, m01); P[1] = pk_bc_s<0>(P[1], t2, m23);
          P[2] = pk_bc_s<1>(P[2], t0, m01);  P[2] = pk_bc_s<0>(P[2], t1, m23); P[2] = pk_bc_s<1>(P[2], t2, m23);
          P[3] = pk_bc_s<0>(P[3], t0, m23);  P[3] = pk_bc_s<1>(P[3], t1, m23); P[3] = pk_bc_s<0>(P[3], t2, p2);
        }
        if constexpr (doS) {
          const float a0 = w0[r * 3], a1 = w0[r * 3 + 1], a2 = w0[r * 3 + 2];
          S01.x = sfma_s(S01.x, a0, n2.y);
          S01.y = sfma_s(S01.y, a0, m[0]);
          S23.x = sfma_s(S23.x, a0, m[1]);
          S23.y = sfma_s(S23.y, a0, m[2]);
          S01 = pfma(f2{a1, a1}, m01, S01);
          S23 = pfma(f2{a1, a1}, m23, S23);
          S01.x = sfma_s(S01.x, a2, m[1]);
          S01.y = sfma_s(S01.y, a2, m[2]);
          S23.x = sfma_s(S23.x, a2, m[3]);
          S23.y = sfma_s(S23.y, a2, p2.x);
        }
      }
    }
    if constexpr (fin) {
      const f4 o = {P[0].x, P[1].x, P[2].x, P[3].x};
      const int zf = zi - 1;
      const unsigned off = zf < b.z1 ? qoff + (unsigned)((long long)zf * HW * (long long)sizeof(T)) : 0x80000000u;
      if constexpr (BH) {
        const b4_t ob = __builtin_convertvector(o, b4_t);
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, ob), yr, off, 0, kDwfAux);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f4, o), yr, off, 0, kDwfAux);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) pin(P[i]);
    pin(S01);
    pin(S23);
    P[0] = f2{P[0].y, S01.x};
    P[1] = f2{P[1].y, S01.y};
    P[2] = f2{P[2].y, S23.x};
    P[3] = f2{P[3].y, S23.y};
    S01 = S23 = zero2;
  };
  run_steps(step, std::make_integer_sequence<int, TZC + 2>{});
}

// ------------------------------------------------------------------------------------------------
// Whole-volume variants for small planes/volumes (the 12^3 and 6^3 levels): one workgroup per
// (n, c) holds the whole zero-padded volume [(D+2)(H+2)(W+2)] in LDS and each thread computes
// voxels v = tid, tid + 256, ... with all 27 taps read straight from LDS.  One load phase and
// one barrier instead of a chain of plane steps: these volumes are latency-, not
// bandwidth-bound.  nchunk = 1 (one partial per (n, c)).
// ------------------------------------------------------------------------------------------------
constexpr int kVolMax = 600;   // measured: the 6^3 level gains, at 12^3 the plane kernels are faster
bool use_volume(int D, int H, int W) { return (long long)(D + 2) * (H + 2) * (W + 2) <= kVolMax; }

// The padded LDS image of volume `src` (transformed if XF; the halo is zero) for the 256-thread
// whole-volume kernels (padded volume <= kVolMax), in two phases: v_fetch issues every load
// of the thread's slots at once (raw values; it does not wait on the InstanceNorm record, so it
// goes before the record merge), v_put transforms and writes them.
constexpr int kVR = (kVolMax + 255) / 256;
template <typename T>
L3U_DEV void v_fetch(float (&raw)[kVR], const T* __restrict__ src, int D, int H, int W) {
  const int PW = W + 2, PH = H + 2, PV = (D + 2) * PH * PW;
#pragma unroll
  for (int r = 0; r < kVR; ++r) {
    const int i = threadIdx.x + 256 * r;
    const int x = i % PW - 1, t = i / PW, y = t % PH - 1, z = t / PH - 1;
    raw[r] = 0.f;
    if (i < PV && x >= 0 && x < W && y >= 0 && y < H && z >= 0 && z < D)
      raw[r] = ld1(src + ((long long)z * H + y) * W + x);
  }
}
template <bool XF>
L3U_DEV void v_put(float* L, const float (&raw)[kVR], int D, int H, int W, float sc, float mu,
                   float sh) {
  const int PW = W + 2, PH = H + 2, PV = (D + 2) * PH * PW;
#pragma unroll
  for (int r = 0; r < kVR; ++r) {
    const int i = threadIdx.x + 256 * r;
    if (i < PV) {
      const int x = i % PW - 1, t = i / PW, y = t % PH - 1, z = t / PH - 1;
      float v = 0.f;
      if (x >= 0 && x < W && y >= 0 && y < H && z >= 0 && z < D) {
        v = raw[r];
        if (XF) v = lrelu(fmaf(sc, v - mu, sh));
      }
      L[i] = v;
    }
  }
}

// y = conv(x) (EPI 0, taps as given) or the data gradient (EPI 1: dpre epilogue + IN sums,
// 2: y += conv^T, 3: y = conv^T; flipped taps), one (n, c) per workgroup
template <typename T, int XF, int EPI>
__global__ __launch_bounds__(256) void dwv_fwd_kernel(
    const T* __restrict__ x, long long xns, const float* __restrict__ w,
    const float* __restrict__ rec, l3u_norm_src src, int has_src, T* __restrict__ y,
    long long yns, const T* __restrict__ ep, long long epns, double* __restrict__ in_part,
    int N, int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(206);
  constexpr bool FLIP = EPI != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nc = blockIdx.x, c = nc % C, n = nc / C;
  const long long HW = (long long)H * W, S = D * HW, cofs = (long long)c * S;
  // wave 0 requests the record's partials and inputs (vector loads, common.h vld) FIRST, then
  // every thread its data, then the taps (scalar loads): one memory round trip for all of them,
  // and the record merge needs only the loads ahead of the data (vector loads complete in order)
  RecPre rp;
  const bool mrg = (XF || EPI == 1) && has_src;
  if (mrg && threadIdx.x < 64) record_pre(src, n, c, C, rp);
  float raw[kVR];
  v_fetch(raw, x + (long long)n * xns + cofs, D, H, W);
  __builtin_amdgcn_sched_barrier(0);
  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + (FLIP ? 26 - t : t)];
  float sc = 1.f, sh = 0.f, mu = 0.f, rstd = 1.f, kk = 1.f;
  if (XF || EPI == 1) {
    if (has_src) {   // (per-wave merges measured +0.2..0.4 us at 6^3: wave 0 merges, LDS broadcast)
      float* s8 = lds;
      if (threadIdx.x < 64) {
        float r[kRec];
        record_finish(src, rp, n, c, C, r);
        if (threadIdx.x == 0) {
#pragma unroll
          for (int i = 0; i < kRec; ++i) s8[i] = r[i];
          if (src.rec_out) {
            float* o = src.rec_out + (long long)nc * kRec;
#pragma unroll
            for (int i = 0; i < kRec; ++i) o[i] = r[i];
          }
        }
      }
      __syncthreads();
      mu = s8[0]; rstd = s8[1]; sc = s8[2]; sh = s8[3]; kk = s8[4];
      __syncthreads();
    } else {
      const float* r = rec + (long long)nc * kRec;
      mu = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4];
    }
  }
  L3U_STAMP_MARK(0);
  v_put<XF == 1>(lds, raw, D, H, W, sc, mu, sh);
  __syncthreads();
  L3U_STAMP_MARK(1);
  const int PW = W + 2, PHW = (H + 2) * PW;
  T* yp = y + (long long)n * yns + cofs;
  const T* epp = (EPI == 1 || EPI == 2) ? ep + (long long)n * epns + cofs : nullptr;
  float s1 = 0.f, s2 = 0.f;
  for (int v = threadIdx.x; v < S; v += blockDim.x) {
    const int xx = v % W, t = v / W, yy = t % H, zz = t / H;
    const float* b = lds + zz * PHW + yy * PW + xx;   // corner of the 3x3x3 neighbourhood
    float o = 0.f;
#pragma unroll
    for (int dz = 0; dz < 3; ++dz)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) o = fmaf(wk[dz * 9 + dy * 3 + dx], b[dz * PHW + dy * PW + dx], o);
    if (EPI == 1) {
      const float e = ld1(epp + v);
      const float pre = fmaf(sc, e - mu, sh);
      o = o * kk * lrelu_d(pre);
      s1 += o;
      s2 += o * ((e - mu) * rstd);
    } else if (EPI == 2) {
      o += ld1(epp + v);
    }
    st1(yp + v, o);
  }
  if (EPI == 1) {
    __syncthreads();
    double* redd = reinterpret_cast<double*>(lds);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, nw = blockDim.x >> 6;
    const double r1 = wave_sum_d((double)s1), r2 = wave_sum_d((double)s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
    __syncthreads();
    if (threadIdx.x < 2) {
      double r = 0.0;
      for (int k = 0; k < nw; ++k) r += redd[k * 2 + threadIdx.x];
      in_part[((long long)c * N + n) * 2 + threadIdx.x] = r;
    }
  }
}

// Both backward halves of the whole-volume form in ONE launch (6^3 level, where each launch is
// latency): the (n, c) volumes of dZ and of A (= x, or lrelu(IN(x)) in MODE 1) sit in LDS side
// by side; each thread forms the flipped-tap data gradient of its voxels (MODE 1: the IN-fused
// dpre epilogue and IN sums; 2: accumulate; 0: overwrite) and the 27 weight-gradient products.
// Same per-voxel arithmetic as dwv_fwd_kernel<0, EPI> + dwv_dw_kernel<XF>.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void dwv_bwd_kernel(
    const float* __restrict__ dz, long long dzns, const T* __restrict__ x, long long xns,
    const float* __restrict__ w, const float* __restrict__ rec, float* __restrict__ dx,
    long long dxns, float* __restrict__ dw_part, double* __restrict__ in_part, int N, int C, int D,
    int H, int W) {
  L3U_STAMP_SCOPE(207);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nc = blockIdx.x, c = nc % C, n = nc / C;
  const long long HW = (long long)H * W, S = D * HW, cofs = (long long)c * S;
  const int PW = W + 2, PHW = (H + 2) * PW, PV = (D + 2) * PHW;
  // both volumes' loads in flight together, ahead of the weights and the IN record
  float rz[kVR], ra[kVR];
  v_fetch(rz, dz + (long long)n * dzns + cofs, D, H, W);
  v_fetch(ra, x + (long long)n * xns + cofs, D, H, W);
  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + 26 - t];
  float sc = 1.f, sh = 0.f, mu = 0.f, rstd = 1.f, kk = 1.f;
  if (MODE == 1) {
    const float* r = rec + (long long)nc * kRec;
    mu = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4];
  }
  float* dzl = lds;
  float* al = lds + PV;
  v_put<false>(dzl, rz, D, H, W, 1.f, 0.f, 0.f);
  v_put<MODE == 1>(al, ra, D, H, W, sc, mu, sh);
  __syncthreads();
  const T* xp = x + (long long)n * xns + cofs;
  float* dxp = dx + (long long)n * dxns + cofs;
  float gw[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) gw[t] = 0.f;
  float s1 = 0.f, s2 = 0.f;
  for (int v = threadIdx.x; v < S; v += blockDim.x) {
    const int xx = v % W, t1 = v / W, yy = t1 % H, zz = t1 / H;
    const int corner = zz * PHW + yy * PW + xx;
    const float* bz = dzl + corner;
    const float* ba = al + corner;
    float o = 0.f;
#pragma unroll
    for (int dzz = 0; dzz < 3; ++dzz)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx)
          o = fmaf(wk[dzz * 9 + dy * 3 + dxx], bz[dzz * PHW + dy * PW + dxx], o);
    const float g = bz[PHW + PW + 1];   // dZ(v)
#pragma unroll
    for (int dzz = 0; dzz < 3; ++dzz)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx) {
          const int tp = dzz * 9 + dy * 3 + dxx;
          gw[tp] = fmaf(g, ba[dzz * PHW + dy * PW + dxx], gw[tp]);
        }
    if (MODE == 1) {
      const float e = ld1(xp + v);
      const float pre = fmaf(sc, e - mu, sh);
      o = o * kk * lrelu_d(pre);
      s1 += o;
      s2 += o * ((e - mu) * rstd);
    } else if (MODE == 2) {
      o += ld1(dxp + v);
    }
    st1(dxp + v, o);
  }
  __syncthreads();
  float* red = lds;                                        // [4 waves][32]
  double* redd = reinterpret_cast<double*>(lds + 4 * 32);  // [4 waves][2]
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    const float r = wave_sum(gw[t]);
    if (ln == 0) red[wv * 32 + t] = r;
  }
  if (MODE == 1) {
    const double r1 = wave_sum_d((double)s1), r2 = wave_sum_d((double)s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
  }
  __syncthreads();
  if (threadIdx.x < 27) {
    float r = 0.f;
    for (int k = 0; k < nw; ++k) r += red[k * 32 + threadIdx.x];
    dw_part[((long long)c * N + n) * 27 + threadIdx.x] = r;
  }
  if (MODE == 1 && threadIdx.x >= 32 && threadIdx.x < 34) {
    const int j = threadIdx.x - 32;
    double r = 0.0;
    for (int k = 0; k < nw; ++k) r += redd[k * 2 + j];
    in_part[((long long)c * N + n) * 2 + j] = r;
  }
}

}  // namespace

#define DW_DISPATCH_P(KERNEL, MODE, ...)                                               \
  do {                                                                                 \
    if (P <= 1) hipLaunchKernelGGL((KERNEL<T, MODE, 1>), __VA_ARGS__);                 \
    else if (P <= 2) hipLaunchKernelGGL((KERNEL<T, MODE, 2>), __VA_ARGS__);            \
    else if (P <= 3) hipLaunchKernelGGL((KERNEL<T, MODE, 3>), __VA_ARGS__);            \
    else if (P <= 4) hipLaunchKernelGGL((KERNEL<T, MODE, 4>), __VA_ARGS__);            \
    else if (P <= 6) hipLaunchKernelGGL((KERNEL<T, MODE, 6>), __VA_ARGS__);            \
    else if (P <= 9) hipLaunchKernelGGL((KERNEL<T, MODE, 9>), __VA_ARGS__);            \
    else if (P <= 12) hipLaunchKernelGGL((KERNEL<T, MODE, 12>), __VA_ARGS__);          \
    else hipLaunchKernelGGL((KERNEL<T, MODE, 16>), __VA_ARGS__);                       \
  } while (0)

namespace {

// the LDS-DMA single-pass backward takes one-wave tiles of <= 128 quads; bf16 moves quad pairs
bool dw_gl(const QGeom& g, int W, int esize) {
  return g.threads == 64 && (g.RB + 2) * g.WQ <= 128 && g.WQ * 4 == W &&
         (esize == 4 || g.WQ % 2 == 0);
}

template <typename T>
int dw3_fwd_impl(const T* x, long long x_nstride, const float* w, const float* rec,
                 const l3u_norm_src* src, T* y, long long y_nstride, int N, int C, int D, int H,
                 int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0);
  const l3u_norm_src z{};
  const l3u_norm_src s = src ? *src : z;
  const int has = src ? 1 : 0;
  const bool xf = rec != nullptr || src != nullptr;
  L3U_REQUIRE(x_nstride >= 0 || (!use_volume(D, H, W) && use_quads(H, W)));
  if (use_volume(D, H, W)) {
    size_t lds = (size_t)(D + 2) * (H + 2) * (W + 2) * sizeof(float);
    if (lds < 16 * sizeof(double)) lds = 16 * sizeof(double);
    if (xf) hipLaunchKernelGGL((dwv_fwd_kernel<T, 1, 0>), dim3(N * C), dim3(256), lds, stream, x, x_nstride, w, rec, s, has, y, y_nstride, nullptr, 0, nullptr, N, C, D, H, W);
    else hipLaunchKernelGGL((dwv_fwd_kernel<T, 0, 0>), dim3(N * C), dim3(256), lds, stream, x, x_nstride, w, rec, s, has, y, y_nstride, nullptr, 0, nullptr, N, C, D, H, W);
    L3U_CHECK_LAUNCH();
  }
  if (use_quads(H, W) && x_nstride % 4 == 0 && y_nstride % 4 == 0) {
    const QGeom g = qgeom(N, C, D, H, W);
    constexpr int E = (int)sizeof(T);
    if (x_nstride < 0) {   // rank-1 input: the fp32 LDS-DMA form with a record only (l3u_dw3_bwd_rank1)
      L3U_REQUIRE(E == 4 && xf && kDwfGl && dw_gl(g, W, E) && (g.RB + 2) * g.WQ > 64);
      const size_t lds = (kDwfPd + 1) * (size_t)(g.RB + 2) * g.WQ * 16 + 8 * sizeof(float);
      dim3 grid(N * C * g.nz * g.ny), block(64);
#define DWGR(T_) hipLaunchKernelGGL((dw3g_fwd_kernel<T, 1, T_, true>), grid, block, lds, stream, x, \
      x_nstride, w, rec, s, has, y, y_nstride, N, C, D, H, W, g.RB, g.RPW, g.ny, g.TZ, g.nz)
      if constexpr (E == 4) { if (g.TZ == 16) DWGR(16); else if (g.TZ == 12) DWGR(12); else if (g.TZ == 8) DWGR(8); else if (g.TZ == 4) DWGR(4); else DWGR(2); }
#undef DWGR
      L3U_CHECK_LAUNCH();
    }
    if (kDwfGl && dw_gl(g, W, E) && (E == 2 || (g.RB + 2) * g.WQ > 64)) {
      // LDS-DMA ring + packed FMAs (dw3g_fwd_kernel)
      const size_t lds = (kDwfPd + 1) * (E == 2 ? (size_t)1024 : (size_t)(g.RB + 2) * g.WQ * 16) + 8 * sizeof(float);
      dim3 grid(N * C * g.nz * g.ny), block(64);
#define DWGF(M_, T_) hipLaunchKernelGGL((dw3g_fwd_kernel<T, M_, T_>), grid, block, lds, stream, x, \
      x_nstride, w, rec, s, has, y, y_nstride, N, C, D, H, W, g.RB, g.RPW, g.ny, g.TZ, g.nz)
      if (xf) { if (g.TZ == 16) DWGF(1, 16); else if (g.TZ == 12) DWGF(1, 12); else if (g.TZ == 8) DWGF(1, 8); else if (g.TZ == 4) DWGF(1, 4); else DWGF(1, 2); }
      else { if (g.TZ == 16) DWGF(0, 16); else if (g.TZ == 12) DWGF(0, 12); else if (g.TZ == 8) DWGF(0, 8); else if (g.TZ == 4) DWGF(0, 4); else DWGF(0, 2); }
#undef DWGF
      L3U_CHECK_LAUNCH();
    }
    size_t lds = (2 * (size_t)(g.RB + 2) * W + 8) * sizeof(float);
    if (lds < 16 * sizeof(double)) lds = 16 * sizeof(double);   // reduction scratch
    dim3 grid(N * C * g.nz * g.ny), block(g.threads);
#define DWQF(M_, T_) hipLaunchKernelGGL((dw3q_fwd_kernel<T, T, M_, 0, T_, kDwqPd>), grid, block, lds, stream, x, \
      x_nstride, w, rec, s, has, y, y_nstride, nullptr, 0, nullptr, N, C, D, H, W, g.RB, g.RPW, \
      g.ny, g.TZ, g.nz)
    if (xf) { if (g.TZ == 16) DWQF(1, 16); else if (g.TZ == 12) DWQF(1, 12); else if (g.TZ == 8) DWQF(1, 8); else if (g.TZ == 4) DWQF(1, 4); else DWQF(1, 2); }
    else { if (g.TZ == 16) DWQF(0, 16); else if (g.TZ == 12) DWQF(0, 12); else if (g.TZ == 8) DWQF(0, 8); else if (g.TZ == 4) DWQF(0, 4); else DWQF(0, 2); }
#undef DWQF
    L3U_CHECK_LAUNCH();
  }
  L3U_REQUIRE(H * W <= 4096);
  const int TZ = pick_tz(D), nchunk = (D + TZ - 1) / TZ;
  const int P = (H * W + 255) / 256;
  const size_t lds = (2 * (size_t)(H + 2) * (W + 2) + 8) * sizeof(float);
  dim3 grid(N * C * nchunk), block(256);
  if (xf) DW_DISPATCH_P(dw3_fwd_kernel, 1, grid, block, lds, stream, x, x_nstride, w, rec, s, has, y, y_nstride, C, D, H, W, TZ, nchunk);
  else DW_DISPATCH_P(dw3_fwd_kernel, 0, grid, block, lds, stream, x, x_nstride, w, rec, s, has, y, y_nstride, C, D, H, W, TZ, nchunk);
  L3U_CHECK_LAUNCH();
}

// data gradient (dx, IN-backward sums) and weight-gradient partials (dw_part) in one call
template <typename T>
int dw3_bwd_impl(const float* dz, long long dz_nstride, const T* x, long long x_nstride,
                 const float* w, const float* rec, float* dx, long long dx_nstride, int accumulate,
                 float* dw_part, double* in_part, int N, int C, int D, int H, int W,
                 hipStream_t stream) {
  constexpr int E = (int)sizeof(T);
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0);
  L3U_REQUIRE(dx != nullptr && dw_part != nullptr);
  L3U_REQUIRE(rec == nullptr || in_part != nullptr);
  L3U_REQUIRE(rec == nullptr || accumulate == 0);
  // a rank-1 input (x_nstride < 0) is taken by the fp32 LDS-DMA single pass with rec only
  const bool xr1 = x_nstride < 0;
  L3U_REQUIRE(!xr1 || (E == 4 && rec != nullptr && !use_volume(D, H, W) && use_quads(H, W) &&
                       dw_gl(qgeom(N, C, D, H, W), W, E)));
  if (use_volume(D, H, W)) {   // data + weight gradient in one launch
    size_t lds2 = 2 * (size_t)(D + 2) * (H + 2) * (W + 2) * sizeof(float);
    if (lds2 < 160 * sizeof(float)) lds2 = 160 * sizeof(float);
#define DWVB(M_) hipLaunchKernelGGL((dwv_bwd_kernel<T, M_>), dim3(N * C), dim3(256), lds2, stream, dz, \
      dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, dw_part, in_part, N, C, D, H, W)
    if (rec) DWVB(1);
    else if (accumulate) DWVB(2);
    else DWVB(0);
#undef DWVB
    L3U_CHECK_LAUNCH();
  }
  if (use_quads(H, W) && x_nstride % 4 == 0 && dz_nstride % 4 == 0 && dx_nstride % 4 == 0) {
    const QGeom g = qgeom(N, C, D, H, W);
    dim3 grid(N * C * g.nz * g.ny), block(g.threads);
    const bool gl = dw_gl(g, W, E);
    // MODE 1 (IN-fused): the LDS-DMA variant, and the register-staged single pass for bf16
    // storage (its 12^3 planes have no bf16 DMA layout: -9 us/step against the split passes);
    // fp32 register-staged measured faster split
    if (rec == nullptr || gl || E == 2) {
      // single pass: data + weight gradient from one read of dZ and A
      size_t lds = 4 * (size_t)(g.RB + 2) * (W + kLPad) * sizeof(float);
      if (lds < 160 * sizeof(float)) lds = 160 * sizeof(float);   // reduction scratch
      if (gl) lds = (kDwgPd + 1) * ((size_t)(g.RB + 2) * g.WQ * 16 + (E == 4 ? (size_t)(g.RB + 2) * g.WQ * 16 : 1024));
#define DWPB(M_, T_) do { if (gl) hipLaunchKernelGGL((dw3p_bwd_kernel<T, M_, T_, true>), grid, block, lds, stream, dz, \
      dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, dw_part, in_part, N, C, D, H, W, g.RB, \
      g.RPW, g.ny, g.TZ, g.nz); \
      else hipLaunchKernelGGL((dw3p_bwd_kernel<T, M_, T_>), grid, block, lds, stream, dz, \
      dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, dw_part, in_part, N, C, D, H, W, g.RB, \
      g.RPW, g.ny, g.TZ, g.nz); } while (0)
#define DWPB_T(M_) do { if (g.TZ == 16) DWPB(M_, 16); else if (g.TZ == 12) DWPB(M_, 12); else if (g.TZ == 8) DWPB(M_, 8); else if (g.TZ == 4) DWPB(M_, 4); else DWPB(M_, 2); } while (0)
      if (xr1) {   // rank-1 input: the LDS-DMA IN-fused variant only (checked above)
        if constexpr (E == 4) {
#define DWPR(T_) hipLaunchKernelGGL((dw3p_bwd_kernel<T, 1, T_, true, true>), grid, block, lds, stream, dz, \
      dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, dw_part, in_part, N, C, D, H, W, g.RB, \
      g.RPW, g.ny, g.TZ, g.nz)
          if (g.TZ == 16) DWPR(16); else if (g.TZ == 12) DWPR(12); else if (g.TZ == 8) DWPR(8); else if (g.TZ == 4) DWPR(4); else DWPR(2);
#undef DWPR
        }
      } else if (rec) DWPB_T(1);
      else if (accumulate) DWPB_T(2);
      else DWPB_T(0);
#undef DWPB_T
#undef DWPB
      L3U_CHECK_LAUNCH();
    }
    // IN-fused on register-staged tiles: the data gradient = the forward stencil with flipped
    // taps and the dpre epilogue, then the weight gradient on its own; both use the same tile
    // geometry, so the chunking of dw_part / in_part is identical to the single pass's
    {
      const l3u_norm_src z{};
      size_t lds = (2 * (size_t)(g.RB + 2) * W + 8) * sizeof(float);
      if (lds < 16 * sizeof(double)) lds = 16 * sizeof(double);
#define DWQX(T_) hipLaunchKernelGGL((dw3q_fwd_kernel<float, T, 0, 1, T_>), grid, block, lds, stream, dz, \
      dz_nstride, w, rec, z, 0, dx, dx_nstride, x, x_nstride, in_part, N, C, D, H, W, g.RB, g.RPW, \
      g.ny, g.TZ, g.nz)
      if (g.TZ == 16) DWQX(16); else if (g.TZ == 12) DWQX(12); else if (g.TZ == 8) DWQX(8); else if (g.TZ == 4) DWQX(4); else DWQX(2);
#undef DWQX
    }
    {
      size_t lds2 = 2 * (size_t)(g.RB + 2) * W * sizeof(float);
      if (lds2 < 128 * sizeof(float)) lds2 = 128 * sizeof(float);
#define DWQW(T_) hipLaunchKernelGGL((dw3q_dw_kernel<T, 1, T_>), grid, block, lds2, stream, dz, \
      dz_nstride, x, x_nstride, rec, dw_part, N, C, D, H, W, g.RB, g.RPW, g.ny, g.TZ, g.nz)
      if (g.TZ == 16) DWQW(16); else if (g.TZ == 12) DWQW(12); else if (g.TZ == 8) DWQW(8); else if (g.TZ == 4) DWQW(4); else DWQW(2);
#undef DWQW
    }
    L3U_CHECK_LAUNCH();
  }
  // small / odd planes: one fused kernel
  L3U_REQUIRE(H * W <= 4096);
  const int TZ = pick_tz(D), nchunk = (D + TZ - 1) / TZ;
  const int P = (H * W + 255) / 256;
  size_t lds = 4 * (size_t)(H + 2) * (W + 2) * sizeof(float);
  if (lds < 128 * sizeof(float)) lds = 128 * sizeof(float);   // reduction scratch
  dim3 grid(N * C * nchunk), block(256);
  if (rec) DW_DISPATCH_P(dw3_bwd_kernel, 1, grid, block, lds, stream, dz, dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, accumulate, dw_part, in_part, N, C, D, H, W, TZ, nchunk);
  else DW_DISPATCH_P(dw3_bwd_kernel, 0, grid, block, lds, stream, dz, dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, accumulate, dw_part, in_part, N, C, D, H, W, TZ, nchunk);
  L3U_CHECK_LAUNCH();
}

}  // namespace

// 1 when l3u_dw3_bwd takes a rank-1 input (x_nstride < 0) with rec at this shape (the fp32
// LDS-DMA single pass, include/l3u.h "Rank-1 operands")
extern "C" int l3u_dw3_bwd_rank1(int N, int C, int D, int H, int W) {
  if (!(N > 0 && C > 0 && !use_volume(D, H, W) && use_quads(H, W))) return 0;
  const QGeom g = qgeom(N, C, D, H, W);
  // the forward's rank-1 form is dw3g_fwd_kernel only (dw3_fwd_impl REQUIREs kDwfGl), with two
  // DMA slots per plane, so a build without it (L3U_DWF_GL=0) offers no rank-1 shape at all
  return dw_gl(g, W, 4) && kDwfGl && (g.RB + 2) * g.WQ > 64;
}

extern "C" int l3u_dw3_nchunk(int N, int C, int D, int H, int W) {
  if (use_volume(D, H, W)) return 1;
  if (use_quads(H, W)) {
    const QGeom g = qgeom(N, C, D, H, W);
    return g.nz * g.ny;
  }
  return (D + pick_tz(D) - 1) / pick_tz(D);
}

#define P_DWF(TT) (const TT* x, long long x_nstride, const float* w, const float* rec,            \
    const l3u_norm_src* src, TT* y, long long y_nstride, int N, int C, int D, int H, int W,          \
    hipStream_t stream)
L3U_TWIN(l3u_dw3_fwd, P_DWF, dw3_fwd_impl(bp(x), x_nstride, w, rec, src, bp(y), y_nstride, N, C, D, H,
         W, stream))
#define P_DWB(TT) (const float* dz, long long dz_nstride, const TT* x, long long x_nstride,        \
    const float* w, const float* rec, float* dx, long long dx_nstride, int accumulate, float* dw_part, \
    double* in_part, int N, int C, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_dw3_bwd, P_DWB, dw3_bwd_impl(dz, dz_nstride, bp(x), x_nstride, w, rec, dx, dx_nstride,
         accumulate, dw_part, in_part, N, C, D, H, W, stream))
