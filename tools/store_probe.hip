// Probe: the cost of a dependent kernel boundary behind a kernel that leaves its output dirty in
// L2 (plain / nt stores) vs written through (sc1 stores), for a 48^3-level tensor (28 MB).
// A graph of REPS x [writer, reader] pairs is replayed; per-pair time by HIP events.
//   hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip -o /tmp/store_probe && /tmp/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void writer(f4* __restrict__ p, const f4* __restrict__ q, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    f4 v = q[i] * 1.0001f;
    if (MODE == 0) {
      p[i] = v;
    } else if (MODE == 1) {
      __builtin_nontemporal_store(v, p + i);
    } else {
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + i), "v"(v) : "memory");
    }
  }
}

__global__ __launch_bounds__(256) void reader(const f4* __restrict__ p, float* __restrict__ out, long n) {
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const f4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
int run(f4* a, f4* b, float* o, long n, int grid, bool with_reader, hipStream_t s) {
  const int REPS = 40;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int r = 0; r < REPS; ++r) {
    hipLaunchKernelGGL(writer<MODE>, dim3(grid), dim3(256), 0, s, a, b, n);
    if (with_reader) hipLaunchKernelGGL(reader, dim3(grid), dim3(256), 0, s, a, o, n);
    else hipLaunchKernelGGL(writer<MODE>, dim3(grid), dim3(256), 0, s, b, a, n);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
  float best = 1e9;
  for (int t = 0; t < 5; ++t) {
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("mode %d %-14s bytes %6.1f MB grid %5d: %7.2f us per pair\n", MODE,
         with_reader ? "write->read" : "write->write", n * 16 / 1e6, grid, 1000.f * best / REPS);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const long nmax = (28311552L / 16) * 2;
  f4 *a, *b;
  float* o;
  CK(hipMalloc(&a, nmax * 16));
  CK(hipMalloc(&b, nmax * 16));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, nmax * 16));
  CK(hipMemset(b, 0, nmax * 16));
  for (long bytes : {1769472L, 7077888L, 28311552L, 56623104L}) {
    const long n = bytes / 16;
    for (int grid : {1024, 4096}) {
      for (int rd = 0; rd < 2; ++rd) {
        if (run<0>(a, b, o, n, grid, rd, s)) return 1;
        if (run<1>(a, b, o, n, grid, rd, s)) return 1;
        if (run<2>(a, b, o, n, grid, rd, s)) return 1;
      }
    }
  }
  return 0;
}
