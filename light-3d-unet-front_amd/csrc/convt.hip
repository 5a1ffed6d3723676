// ConvTranspose3d(Ci, Co, k=2, s=2) backward in ONE pass over the up-sampled gradient (UpBlock.up,
// unet3d.py:119; its autograd backward).  With dY [N][Co][2D][2H][2W] (read in place from the
// decoder's concat gradient), X [N][Ci][D][H][W] the layer input and w [Ci][Co][2][2][2]:
//   dX[ci][z,y,x]      = sum_{co,a,b,c} w[ci][co][a][b][c] dY[co][2z+a][2y+b][2x+c]
//   dW[ci][co][a][b][c] = sum_{n,z,y,x} X[ci][z,y,x] dY[co][2z+a][2y+b][2x+c]
//   db[co]             = sum of dY[co]
// Both GEMMs are K = Co*8 deep per input voxel, so at the 24^3 / 12^3 decoder steps the pass is
// as much MFMA work (2 * 8*Co*Ci MAC per voxel, fp32 MFMA at 157 TFLOP/s) as HBM traffic: dY is
// read ONCE from HBM into LDS and both products are formed from the LDS copy.
//
// Work unit: a tile of P = 16*PB consecutive x-PAIRS of input voxels (pair p = (z*H + y)*W/2 + xp
// holds voxels 2p and 2p+1 of the flattened volume: the two input voxels whose 2x2x2 children share
// the output rows).  For one (co, a, b) the four dY values of a pair -- (2x, c0) (2x, c1)
// (2x+1, c0) (2x+1, c1) -- are ONE contiguous float4 of an up-sampled row, and the pairs of a tile
// are consecutive float4s of those rows: the staging loads are plain coalesced 16-byte loads.
// LDS holds the tile as sdy[co][ab][pair] float4 (row pitch P+1 float4: conflict-free reads in both
// operand layouts) and the input channels of the workgroup as sx[ci][2P voxels] (pitch 2P+4).
// A workgroup (4 waves) covers CIB blocks of 16 input channels of its tiles:
//   data gradient   wave w owns (pair block w % PB, channel block w / PB): per 4 co and (a, b),
//                   lane (lr, lk) reads the float4 of pair 16*pb + lr at co = 4q + lk and feeds
//                   its components into the even / odd voxel accumulators (MFMA 16x16x4: rows =
//                   16 ci, columns = 16 pairs, k = 4 co), the weights as the A operand from
//                   registers (32 per 16 co, loaded once);
//   weight gradient wave w owns CIB of the (channel block, 4-co group) units: the voxel is the MFMA
//                   k-dimension (4 pairs per step), A = X[ci][pair] (a float2: even / odd voxel),
//                   B = the float4 of (co, ab) = column lr at pair lk; the accumulators (16 ci x
//                   16 (co, ab) columns, c = 0 / 1 separately) live across all tiles of the
//                   workgroup and are written once as its partial;
//   bias            the channel-block-0 units also sum their float4s (one partial per workgroup).
// A workgroup takes TPB consecutive tiles; the next tile's loads are issued before the current
// tile's MFMAs (register prefetch), so staging overlaps the math.
#include "common.h"
using namespace l3u;

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

L3U_DEV f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

template <typename T, int CO, int PB, int CIB, int NCS, bool PF = true>
__global__ __launch_bounds__(256) void convt_bwd_tile_kernel(
    const float* __restrict__ dy, long long dyns, const T* __restrict__ x, long long xns,
    const float* __restrict__ w, float* __restrict__ dx, long long dxns, float* __restrict__ wpart,
    float* __restrict__ bpart, int Ci, int D, int H, int W, int ntile, int ntg, int tpb) {
  L3U_STAMP_SCOPE(120);
  static_assert(PB * CIB == 4, "one data-gradient unit per wave");
  constexpr int P = 16 * PB;            // pairs per tile
  constexpr int NCH = CO / 16;          // 16-channel chunks of co
  constexpr int NST = NCH / NCS;        // LDS stages per tile (NCS chunks each)
  static_assert(NST * NCS == NCH, "whole chunks per stage");
  constexpr int RP = P + 1;             // sdy row pitch (float4)
  constexpr int XP = 2 * P + 4;         // sx row pitch (float)
  constexpr int NCI = 16 * CIB;         // input channels of this workgroup
  constexpr int NLD = 16 * NCS * 4 * P / 256;     // dY float4 per thread per stage
  constexpr int NLX = NCI * (2 * P / 4) / 256;    // X float4 per thread per tile
  static_assert(NLD * 256 == 16 * NCS * 4 * P && NLX * 256 == NCI * (2 * P / 4), "staging split");
  static_assert((256 / P) % 4 == 0, "a lane's dY loads share their ab row");
  __shared__ __attribute__((aligned(16))) f4 sdy[16 * NCS * 4 * RP];
  __shared__ __attribute__((aligned(16))) float sx[NCI * XP];

  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, lr = l & 15, lk = l >> 4;
  const int WP = W >> 1, PP = D * H * WP;
  const long long S = (long long)D * H * W, S8 = 8 * S;
  const int bx = blockIdx.x, n = bx / ntg, g = bx % ntg;
  const int ci_wg = blockIdx.y * NCI;
  const int t_lo = g * tpb, t_hi = min(ntile, t_lo + tpb);
  const float* dyn = dy + (long long)n * dyns;
  const T* xn = x + (long long)n * xns;
  const int K = CO * 8;

  // data-gradient unit of this wave and its weights w[ci][co][a][b][c]: lane (lr, lk) holds, per
  // 16-co chunk and co quad q, the 8 taps of (ci = ci0x + lr, co = 16 ch + 4q + lk)
  const int pbx = wave % PB, cbx = wave / PB;
  const int ci0x = ci_wg + 16 * cbx;
  // (the weight is a view into the flat parameter buffer: 4-byte alignment only, hence dword
  // loads; through a descriptor so that the per-chunk offsets are immediates)
  constexpr int NW = NST > 1 ? NCS : NCH;   // chunks of taps held at once
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(w), 0, (int)min((long long)Ci * K * 4, 0x7fffffffll), 0x00020000);
  const unsigned wlane = (unsigned)((ci0x + lr) * K + lk * 8) * 4u;
  auto load_w = [&](float (&dst)[NW][4][8], int ch0) {
#pragma unroll
    for (int cc = 0; cc < NW; ++cc)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          dst[cc][q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
              wrs, wlane + (unsigned)(((16 * (ch0 + cc) + 4 * q) * 8 + e) * 4), 0, 0));
  };
  float wr[NW][4][8], wn[NST > 1 ? NW : 1][4][8];
  load_w(wr, 0);
  // weight-gradient accumulators: unit u = wave * CIB + j -> (channel block u / 4, co group u % 4)
  f4 acc[NCH][CIB][2];
  float bacc[NCH][CIB];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int j = 0; j < CIB; ++j) {
      acc[ch][j][0] = acc[ch][j][1] = f4{0.f, 0.f, 0.f, 0.f};
      bacc[ch][j] = 0.f;
    }

  // ---- staging: thread tid loads dY float4 i*256 + tid = ((co*4 + ab) * P + pair) of the stage's
  // co range and (first stage of a tile) X float4 i*256 + tid = (ci * P/2 + chunk)
  f4 rd[NLD], rx[NLX];
  // a lane's pair within the tile is the same for all its dY loads (256 % P == 0) and its X
  // chunk the same for all its X loads, so the index arithmetic is done once per tile; loads past
  // the volume read a clamped in-range address and are zeroed when they are written to LDS (a
  // select on the loaded value here would wait for the load: the prefetch must stay in flight)
  constexpr int RPT = 256 / P, CPT = 256 / (P / 2);
  const int pr0 = tid % P, xj0 = tid % (P / 2);
  const long long plane2 = 4ll * H * W;   // one up-sampled plane (2H x 2W)
  bool okd = false, okx = false;
  // dY through a buffer descriptor over the sample: the lane's part of the offset (its pair, its
  // (co, ab) row) is one 32-bit VGPR per tile, the per-load part (the co block of load i and of the
  // stage) is wave-uniform and goes in soffset -- flat 64-bit addresses of the NLD loads would be
  // hoisted out of the tile loop and, at Co = 64, spill
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(dyn), 0, (int)min((long long)CO * S8 * 4, 0x7fffffffll), 0x00020000);
  const int rlane = tid / P;   // (co, ab) row of the lane's loads: co = 4 i RPT/4 + rlane / 4
  const unsigned lane_row = (unsigned)((rlane >> 2) * S8 + ((rlane & 3) >> 1) * plane2 + (rlane & 1) * (2 * W)) * 4u;
  auto load_stage = [&](int t, int st) {
    const int pbase = t * P, p = pbase + pr0;
    const bool ok = p < PP;
    okd = ok;
    const int pc = ok ? p : PP - 1;
    const int xp = pc % WP, tt = pc / WP, y = tt % H, z = tt / H;
    const unsigned voff = lane_row + (unsigned)(((2 * z) * (2 * H) + 2 * y) * (2 * W) + 4 * xp) * 4u;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int soff = (int)((long long)(16 * NCS * st + i * (RPT / 4)) * S8 * 4);
      rd[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(dyr, voff, soff, 0));
    }
    if (st == 0) {
      const long long s0 = 2ll * pbase + 4 * xj0;
      const bool xok = s0 < S;
      okx = xok;
      const T* xsrc = xn + (xok ? s0 : 0);
#pragma unroll
      for (int i = 0; i < NLX; ++i) {
        const int ci = i * CPT + tid / (P / 2);
        const f4 v = ldv4(xsrc + (long long)(ci_wg + ci) * S);
        rx[i] = v;
      }
    }
  };
  auto store_stage = [&](int st) {
#pragma unroll
    for (int i = 0; i < NLD; ++i)
      sdy[(i * RPT + tid / P) * RP + pr0] = okd ? rd[i] : f4{0.f, 0.f, 0.f, 0.f};
    if (st == 0) {
#pragma unroll
      for (int i = 0; i < NLX; ++i)
        *reinterpret_cast<f4*>(sx + (i * CPT + tid / (P / 2)) * XP + 4 * xj0) =
            okx ? rx[i] : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // LDS-only workgroup barrier: __syncthreads() would also wait for this wave's global stores and
  // the next tile's prefetch loads (a workgroup-scope fence); only the LDS tile needs ordering here
  auto lds_barrier = [] {
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0); vmcnt / expcnt untouched
    __builtin_amdgcn_s_barrier();
  };

  if (t_lo < t_hi) load_stage(t_lo, 0);
  for (int t = t_lo; t < t_hi; ++t) {
    // data-gradient accumulators of the tile: four independent chains (even / odd voxel x
    // c = 0 / 1, summed at the end) so that back-to-back MFMAs never wait on each other
    f4 ae0 = {0.f, 0.f, 0.f, 0.f}, ae1 = ae0, ao0 = ae0, ao1 = ae0;
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      store_stage(st);
      lds_barrier();
#ifdef L3U_STAMP_CT
      if (st == 0 && t == t_lo) L3U_STAMP_MARK(0);   // stamp variant: the first stage staged
#endif
      if constexpr (NST > 1) __builtin_amdgcn_sched_barrier(0);   // keep the stages apart
      // the next stage's loads (and taps) are in flight during this stage's MFMAs
      if (st + 1 < NST) {
        load_stage(t, st + 1);
      } else if (PF && t + 1 < t_hi) {
        // (PF = false: one tile per workgroup, no next tile; its staging registers are then free
        // during the MFMAs, which lets the LDS operand reads run ahead instead of one at a time)
        load_stage(t + 1, 0);
      }
      if constexpr (NST > 1) load_w(wn, ((st + 1) % NST) * NCS);
      // ---- data gradient: 16 ci x 16 pairs over the stage's co chunks; LDS operands one
      // (chunk, co quad) ahead: 4 reads in flight across each group of 16 MFMAs
      f4 vn[4];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) vn[ab] = sdy[(lk * 4 + ab) * RP + 16 * pbx + lr];
#pragma unroll
      for (int cq = 0; cq < 4 * NCS; ++cq) {
        const int cc = cq >> 2, q = cq & 3;
        f4 v[4];
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) v[ab] = vn[ab];
        if (cq + 1 < 4 * NCS) {
#pragma unroll
          for (int ab = 0; ab < 4; ++ab) vn[ab] = sdy[((4 * (cq + 1) + lk) * 4 + ab) * RP + 16 * pbx + lr];
        }
        // the reads above stay ahead of this quad's MFMAs (left to itself the scheduler issued each
        // read right before its four MFMAs and waited for it: one LDS latency per read, at one
        // wave per SIMD nothing hides it)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) {
          const float* wq = wr[NST > 1 ? cc : st * NCS + cc][q];
          ae0 = mfma4(wq[2 * ab], v[ab][0], ae0);
          ae1 = mfma4(wq[2 * ab + 1], v[ab][1], ae1);
          ao0 = mfma4(wq[2 * ab], v[ab][2], ao0);
          ao1 = mfma4(wq[2 * ab + 1], v[ab][3], ao1);
        }
      }
      // ---- weight gradient (+ bias): the voxel pair is the k-dimension, 4 pairs per step
#pragma unroll
      for (int j = 0; j < CIB; ++j) {
        const int u = wave * CIB + j, cb = u >> 2, gq = u & 3;
        const float* sxr = sx + (16 * cb + lr) * XP;
#pragma unroll
        for (int cc = 0; cc < NCS; ++cc) {
          const int ch = st * NCS + cc;
          const f4* srow = sdy + (64 * cc + 16 * gq + lr) * RP;   // (co*4 + ab) = 16 (4cc + gq) + lr
#pragma unroll
          for (int kp = 0; kp < P / 4; ++kp) {
            const f4 v = srow[4 * kp + lk];
            const f2_t xv = *reinterpret_cast<const f2_t*>(sxr + 2 * (4 * kp + lk));
            acc[ch][j][0] = mfma4(xv[0], v[0], acc[ch][j][0]);
            acc[ch][j][1] = mfma4(xv[0], v[1], acc[ch][j][1]);
            acc[ch][j][0] = mfma4(xv[1], v[2], acc[ch][j][0]);
            acc[ch][j][1] = mfma4(xv[1], v[3], acc[ch][j][1]);
            if (cb == 0) bacc[ch][j] += (v[0] + v[1]) + (v[2] + v[3]);
          }
        }
      }
      if (st + 1 == NST) {
        // ---- store the tile's data gradient: ci = ci0x + 4 lk + r, pair = tile pair 16 pbx + lr
        const f4 ae = ae0 + ae1, ao = ao0 + ao1;
        const int p = t * P + 16 * pbx + lr;
        if (p < PP) {
          float* dxn = dx + (long long)n * dxns + 2ll * p;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            *reinterpret_cast<f2_t*>(dxn + (long long)(ci0x + 4 * lk + r) * S) = f2_t{ae[r], ao[r]};
        }
      }
      if constexpr (NST > 1) {
#pragma unroll
        for (int cc = 0; cc < NW; ++cc)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) wr[cc][q][e] = wn[cc][q][e];
      }
      lds_barrier();   // sdy / sx are rewritten by the next stage
    }
  }
#ifdef L3U_STAMP_CT
  L3U_STAMP_MARK(1);   // stamp variant: every tile's MFMAs issued
#endif
  // ---- weight-gradient partial of this workgroup: part[bx][ci][co*8 + 4a + 2b + c]
  float* o = wpart + (long long)bx * Ci * K;
#pragma unroll
  for (int j = 0; j < CIB; ++j) {
    const int u = wave * CIB + j, cb = u >> 2, gq = u & 3;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ci = ci_wg + 16 * cb + 4 * lk + r, co = 16 * ch + 4 * gq + (lr >> 2);
          o[(long long)ci * K + co * 8 + 2 * (lr & 3) + c] = acc[ch][j][c][r];
        }
  }
  // ---- bias partial: lanes of one co are (lr & 3) x lk; fixed xor order
  if (bpart != nullptr && blockIdx.y == 0) {
#pragma unroll
    for (int j = 0; j < CIB; ++j) {
      const int u = wave * CIB + j, cb = u >> 2, gq = u & 3;
      if (cb != 0) continue;   // wave-uniform
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        float bv = bacc[ch][j];
        bv += __shfl_xor(bv, 1, 64);
        bv += __shfl_xor(bv, 2, 64);
        bv += __shfl_xor(bv, 16, 64);
        bv += __shfl_xor(bv, 32, 64);
        if (l < 16 && (lr & 3) == 0) bpart[(long long)bx * CO + 16 * ch + 4 * gq + (lr >> 2)] = bv;
      }
    }
  }
}

}  // namespace

namespace l3u {

// The tile shape for (Ci, Co, D, H, W): PB pair blocks, CIB channel blocks per workgroup, TPB
// tiles per workgroup; false when the tile kernel does not take the shape.
struct ConvtTile { int pb, cib, tpb, ntile, ntg; };
static bool convt_tile_shape(int N, int Ci, int Co, int D, int H, int W, ConvtTile& t) {
  if (!(N > 0 && D > 0 && H > 0 && W > 0 && (Co == 16 || Co == 32 || Co == 64) && Ci % 16 == 0))
    return false;
  const long long S = (long long)D * H * W;
  if (W % 2 != 0 || S % 4 != 0 || S > (1ll << 26)) return false;
  // dY is read through a buffer descriptor over one sample (32-bit num_records, voffset and
  // soffset): every byte offset of the sample's Co * 8 * S floats must stay below 2^31, otherwise
  // the loads past the limit return 0 silently (the three-launch path takes such volumes)
  if ((long long)Co * 32 * S >= (1ll << 31)) return false;
  const int PP = D * H * (W / 2);
  // 16 input channels per block; 2 blocks per workgroup (up to 32 channels) with 32-pair tiles,
  // 4 blocks with 16-pair tiles for the wider layers (same LDS footprint) when the volume has
  // tiles enough for several per workgroup; a small wide layer (the 12^3 up2) takes one block per
  // workgroup over 64-pair tiles instead: the same time (tools/pwbench.py --convt-only, 12.5 vs
  // 12.1 us) with a quarter of the weight-partial bytes (3.5 vs 14 MB at 12^3)
  // Co = 64 (config 5's 16^3 up2): one block over 64-pair tiles, staged one 16-co chunk at a
  // time; only for volumes with 64 tiles at least (at 6^3 the three-launch form is 3x faster)
  const int PP0 = D * H * (W / 2);
  if (Co == 64 && (long long)N * PP0 < 4096) return false;
  if (Co == 64) { t.pb = 4; t.cib = 1; }
  else if (Ci % 64 == 0 && (long long)N * ((PP0 + 15) / 16) >= 1024) { t.pb = 1; t.cib = 4; }
  else if (Ci % 32 == 0 && Ci % 64 != 0) { t.pb = 2; t.cib = 2; }
  else { t.pb = 4; t.cib = 1; }
  const int P = 16 * t.pb;
  t.ntile = (PP + P - 1) / P;
  // tiles per workgroup: as many as keep >= 256 workgroups (one per CU at least); each workgroup
  // writes one weight partial, so fewer workgroups = fewer partial bytes
  const long long units = (long long)N * t.ntile * (Ci / (16 * t.cib));
  t.tpb = 1;
  while (t.tpb < 16 && units / (2 * t.tpb) >= 256) t.tpb *= 2;
  t.ntg = (t.ntile + t.tpb - 1) / t.tpb;
  return true;
}

int convt_tile_nparts(int N, int Ci, int Co, int D, int H, int W) {
  ConvtTile t;
  return convt_tile_shape(N, Ci, Co, D, H, W, t) ? N * t.ntg : 0;
}

template <typename T>
int convt_tile_launch(const float* dy, long long dy_nstride, const T* x, long long x_nstride,
                      const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                      int N, int Ci, int Co, int D, int H, int W, hipStream_t stream) {
  ConvtTile t;
  L3U_REQUIRE(convt_tile_shape(N, Ci, Co, D, H, W, t) && dy && x && w && dx && wpart);
  L3U_REQUIRE(((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 7) == 0 &&
              ((uintptr_t)x & (4 * sizeof(T) - 1)) == 0 && dy_nstride % 4 == 0 && x_nstride % 4 == 0 &&
              dx_nstride % 2 == 0);
  dim3 grid(N * t.ntg, Ci / (16 * t.cib)), block(256);
#define CTT0(CO_, PB_, CIB_, PF_) hipLaunchKernelGGL((convt_bwd_tile_kernel<T, CO_, PB_, CIB_, (CO_ == 64 ? 1 : CO_ / 16), PF_>), \
    grid, block, 0, stream, dy, dy_nstride, x, x_nstride, w, dx, dx_nstride, wpart, bpart, Ci, D, H, W, t.ntile, t.ntg, t.tpb)
#define CTT(CO_, PB_, CIB_) do { if (t.tpb > 1) CTT0(CO_, PB_, CIB_, true); else CTT0(CO_, PB_, CIB_, false); } while (0)
  if (Co == 64) {
    CTT(64, 4, 1);
  } else if (Co == 16) {
    if (t.cib == 4) CTT(16, 1, 4); else if (t.cib == 2) CTT(16, 2, 2); else CTT(16, 4, 1);
  } else {
    if (t.cib == 4) CTT(32, 1, 4); else if (t.cib == 2) CTT(32, 2, 2); else CTT(32, 4, 1);
  }
#undef CTT
#undef CTT0
  L3U_CHECK_LAUNCH();
}

template int convt_tile_launch<float>(const float*, long long, const float*, long long, const float*,
                                      float*, long long, float*, float*, int, int, int, int, int, int,
                                      hipStream_t);
template int convt_tile_launch<bf16>(const float*, long long, const bf16*, long long, const float*,
                                     float*, long long, float*, float*, int, int, int, int, int, int,
                                     hipStream_t);

}  // namespace l3u
