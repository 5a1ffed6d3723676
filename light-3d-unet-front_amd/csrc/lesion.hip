// Lesion post-processing on the device: connected-component labelling and per-component
// statistics.  Replaces the host scipy/numpy work of
//   light_unet/models/metrics.py:38-63   get_connected_components (ndimage.label with its default
//                                        structure: face connectivity in every dimension of the
//                                        array -- 6 neighbours for a [D, H, W] volume, 8 for a
//                                        batched [B, D, H, W] array, where the same voxel of
//                                        consecutive batch items is connected; min_size filter +
//                                        relabel)
//   light_unet/models/metrics.py:107-213 component centres of mass, pairwise overlap (IoU) counts
//   light_unet/core/inferencer.py:62-111 bounding boxes, volumes and peak probability per component
// (host-bound with real volumes).  Integer work, bit-exact:
//   * labelling: lock-free union-find over the face neighbours (atomicMin links every root to the
//     SMALLER linear index, so the final root of a component is its first voxel in raster order);
//     components are then numbered by the rank of that first voxel (a chunk-count + scan +
//     ballot-ranked scatter), which is exactly scipy.ndimage.label's numbering (order of first
//     encounter in a C-order scan);
//   * statistics: 64-bit integer atomics (sizes, coordinate sums, bounding boxes) and the peak
//     probability as the max of non-negative float bit patterns (order-preserving), so no result
//     depends on the order in which workgroups arrive.
#include "common.h"
using namespace l3u;

namespace {

L3U_DEV int uf_find(const int* __restrict__ parent, int x) {
  int p = parent[x];
  while (p != x) {
    x = p;
    p = parent[x];
  }
  return x;
}

// every foreground voxel starts as its own root; -1 = background
__global__ __launch_bounds__(256) void ccl_init_kernel(const float* __restrict__ src, float thr,
                                                       int* __restrict__ parent, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    parent[i] = src[i] >= thr ? (int)i : -1;
}

// union of a and b: link the larger root under the smaller one (atomicMin keeps parent[x] <= x,
// so every path strictly decreases and the walk terminates)
L3U_DEV void uf_union(int* parent, int a, int b) {
  while (true) {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    if (a == b) return;
    if (a < b) { const int t = a; a = b; b = t; }   // a > b: a becomes a child of b
    const int old = atomicMin(&parent[a], b);
    if (old == a) return;                            // a was still a root: linked
    a = old;                                         // linked elsewhere meanwhile: retry
  }
}

// face neighbours of [B][D][H][W]: x, y, z within an item and b (the same voxel of the previous
// item, offset S = D*H*W) -- ndimage.label's default structure for a 4-dimensional array
__global__ __launch_bounds__(256) void ccl_merge_kernel(int* __restrict__ parent, int B, int D, int H,
                                                        int W) {
  const long long S = (long long)D * H * W, n = B * S, HW = (long long)H * W;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    if (parent[i] < 0) continue;
    const long long r = i % S;
    const int x = (int)(r % W), y = (int)((r / W) % H), z = (int)(r / HW);
    if (x > 0 && parent[i - 1] >= 0) uf_union(parent, (int)i, (int)(i - 1));
    if (y > 0 && parent[i - W] >= 0) uf_union(parent, (int)i, (int)(i - W));
    if (z > 0 && parent[i - HW] >= 0) uf_union(parent, (int)i, (int)(i - HW));
    if (i >= S && parent[i - S] >= 0) uf_union(parent, (int)i, (int)(i - S));
  }
}

// parent[i] = root(i); count[c] = roots in chunk c (kCh voxels per chunk)
constexpr int kCh = 4096;
__global__ __launch_bounds__(256) void ccl_flatten_kernel(int* __restrict__ parent, long long n,
                                                          int* __restrict__ count) {
  __shared__ int red[4];
  const long long b0 = (long long)blockIdx.x * kCh;
  int c = 0;
  for (int k = threadIdx.x; k < kCh; k += 256) {
    const long long i = b0 + k;
    if (i < n && parent[i] >= 0) {
      const int r = uf_find(parent, (int)i);
      parent[i] = r;
      c += r == (int)i;
    }
  }
  c = (int)wave_sum((float)c);   // <= 4096: exact in fp32
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) count[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// exclusive scan of the chunk counts (one workgroup, any length); the total lands in count[nb]
__global__ __launch_bounds__(256) void ccl_scan_kernel(int* __restrict__ count, int nb) {
  __shared__ int part[256];
  const int per = (nb + 255) / 256, lo = threadIdx.x * per, hi = min(nb, lo + per);
  int s = 0;
  for (int i = lo; i < hi; ++i) s += count[i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    for (int t = 0; t < 256; ++t) { const int v = part[t]; part[t] = a; a += v; }
    count[nb] = a;
  }
  __syncthreads();
  int a = part[threadIdx.x];
  for (int i = lo; i < hi; ++i) { const int v = count[i]; count[i] = a; a += v; }
}

// roots get their label, 1 + their rank in raster order: ballot ranks inside each round of 256
// consecutive voxels, rounds in order
__global__ __launch_bounds__(256) void ccl_root_label_kernel(const int* __restrict__ parent,
                                                             long long n,
                                                             const int* __restrict__ offs,
                                                             int* __restrict__ label) {
  __shared__ int wsum[4];
  __shared__ int base;
  const long long b0 = (long long)blockIdx.x * kCh;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (threadIdx.x == 0) base = offs[blockIdx.x];
  __syncthreads();
  for (int k0 = 0; k0 < kCh; k0 += 256) {
    const long long i = b0 + k0 + threadIdx.x;
    const bool root = i < n && parent[i] == (int)i;
    const unsigned long long m = __ballot(root);
    const int before = __popcll(m & ((1ull << ln) - 1ull));
    if (ln == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int pre = base;
    for (int w = 0; w < wv; ++w) pre += wsum[w];
    if (root) label[i] = pre + before + 1;
    __syncthreads();
    if (threadIdx.x == 0) base += (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void ccl_label_kernel(const int* __restrict__ parent,
                                                        int* __restrict__ label, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int p = parent[i];
    if (p < 0) label[i] = 0;
    else if (p != (int)i) label[i] = label[p];
  }
}

// per component l (1-based): stats[(l-1)*12 + k], k = 0 size, 1..3 sum of the three leading
// coordinates (c0, c1, c2), 4..6 their minima, 7..9 their maxima, 10 max prob (float bits;
// prob >= 0).  The leading coordinates are (z, y, x) of a 3-dimensional array and (b, z, y) of a
// 4-dimensional one (lead4): the reference keeps the first three of ndimage.center_of_mass's
// coordinates whatever the rank (metrics.py:99-124).  remap (optional) renumbers the labels in
// place first (0 drops the voxel).
__global__ __launch_bounds__(256) void ccl_stats_kernel(int* __restrict__ label,
                                                        const int* __restrict__ remap,
                                                        const float* __restrict__ prob,
                                                        unsigned long long* __restrict__ stats,
                                                        int B, int D, int H, int W, int lead4) {
  const long long S = (long long)D * H * W, n = B * S, HW = (long long)H * W;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    int l = label[i];
    if (l <= 0) continue;
    if (remap) {
      l = remap[l];
      label[i] = l;
      if (l <= 0) continue;
    }
    const long long r = i % S;
    const unsigned long long x = r % W, y = (r / W) % H, z = r / HW, b = i / S;
    const unsigned long long c0 = lead4 ? b : z, c1 = lead4 ? z : y, c2 = lead4 ? y : x;
    unsigned long long* s = stats + (long long)(l - 1) * 12;
    atomicAdd(s + 0, 1ull);
    atomicAdd(s + 1, c0);
    atomicAdd(s + 2, c1);
    atomicAdd(s + 3, c2);
    atomicMin(s + 4, c0);
    atomicMin(s + 5, c1);
    atomicMin(s + 6, c2);
    atomicMax(s + 7, c0);
    atomicMax(s + 8, c1);
    atomicMax(s + 9, c2);
    if (prob) atomicMax(s + 10, (unsigned long long)__float_as_uint(fmaxf(prob[i], 0.f)));
  }
}

__global__ __launch_bounds__(256) void ccl_stats_init_kernel(unsigned long long* __restrict__ stats,
                                                             int ncomp) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < ncomp * 12; i += gridDim.x * 256) {
    const int k = i % 12;
    stats[i] = (k >= 4 && k <= 6) ? ~0ull : 0ull;
  }
}

// overlap counts of two labellings: inter[a * (nb + 1) + b] += 1 where both labels are > 0
__global__ __launch_bounds__(256) void ccl_pairs_kernel(const int* __restrict__ la,
                                                        const int* __restrict__ lb, int nb,
                                                        unsigned int* __restrict__ inter,
                                                        long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int a = la[i], b = lb[i];
    if (a > 0 && b > 0) atomicAdd(inter + (long long)a * (nb + 1) + b, 1u);
  }
}

int blocks_for(long long n) {
  const long long b = (n + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

int l3u_ccl_nchunks(long long n) { return (int)((n + kCh - 1) / kCh); }

int l3u_ccl_label_b(const float* src, float threshold, int* parent, int* label, int* chunk_count,
                    int B, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(src && parent && label && chunk_count && B > 0 && D > 0 && H > 0 && W > 0);
  const long long n = (long long)B * D * H * W;
  L3U_REQUIRE(n < (1ll << 31));
  const int nb = l3u_ccl_nchunks(n);
  hipLaunchKernelGGL(ccl_init_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, src, threshold,
                     parent, n);
  hipLaunchKernelGGL(ccl_merge_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, parent, B, D, H, W);
  hipLaunchKernelGGL(ccl_flatten_kernel, dim3(nb), dim3(256), 0, stream, parent, n, chunk_count);
  hipLaunchKernelGGL(ccl_scan_kernel, dim3(1), dim3(256), 0, stream, chunk_count, nb);
  hipLaunchKernelGGL(ccl_root_label_kernel, dim3(nb), dim3(256), 0, stream, parent, n, chunk_count,
                     label);
  hipLaunchKernelGGL(ccl_label_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, parent, label, n);
  L3U_CHECK_LAUNCH();
}

int l3u_ccl_label(const float* src, float threshold, int* parent, int* label, int* chunk_count,
                  int D, int H, int W, hipStream_t stream) {
  return l3u_ccl_label_b(src, threshold, parent, label, chunk_count, 1, D, H, W, stream);
}

int l3u_ccl_stats_b(int* label, const int* remap, const float* prob, unsigned long long* stats,
                    int ncomp, int B, int D, int H, int W, int lead4, hipStream_t stream) {
  L3U_REQUIRE(label && stats && ncomp > 0 && B > 0 && D > 0 && H > 0 && W > 0);
  L3U_REQUIRE(lead4 == 0 ? B == 1 : lead4 == 1);
  const long long n = (long long)B * D * H * W;
  hipLaunchKernelGGL(ccl_stats_init_kernel, dim3(blocks_for(ncomp * 12ll)), dim3(256), 0, stream,
                     stats, ncomp);
  hipLaunchKernelGGL(ccl_stats_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, label, remap,
                     prob, stats, B, D, H, W, lead4);
  L3U_CHECK_LAUNCH();
}

int l3u_ccl_stats(int* label, const int* remap, const float* prob, unsigned long long* stats,
                  int ncomp, int D, int H, int W, hipStream_t stream) {
  return l3u_ccl_stats_b(label, remap, prob, stats, ncomp, 1, D, H, W, 0, stream);
}

int l3u_ccl_pairs(const int* label_a, const int* label_b, int nb, unsigned int* inter, long long n,
                  hipStream_t stream) {
  L3U_REQUIRE(label_a && label_b && inter && nb >= 0 && n > 0);
  hipLaunchKernelGGL(ccl_pairs_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, label_a, label_b,
                     nb, inter, n);
  L3U_CHECK_LAUNCH();
}

}  // extern "C"
