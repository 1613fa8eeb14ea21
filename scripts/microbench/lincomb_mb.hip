// theta-lincomb microbenchmark (C3 multi-query: out[s] = sum_q theta[s][q] v_q, 2 components of 75.46 M
// doubles, 128 samples = 77 GB written).  Variants of the write organisation:
//   pers32  : production (hdd_affine_lincomb): persistent grid-stride 256-thread WGs, 32 samples per launch,
//             each lane 16 B per sample (nt or plain stores)
//   pers128 : the same with all 128 samples in one launch (components read once; theta in LDS)
//   nonp32  : one 4 KB chunk (256 lanes x 16 B) per workgroup, 32 samples per launch
//   blocked : sample-major inside blocks of B values: workgroup (block, sample, chunk) in dispatch order, so the
//             concurrently written addresses form one contiguous window of one sample (fill-like); the
//             block's components (2 x B x 8 bytes) are re-read per sample from L2 / MALL
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result lincomb_mb.hip -o lincomb_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));

struct Args {
  const double* v0;
  const double* v1;
  double* out;
  const double* theta;   // [128][2]
  long nnz, stride;
  int s0, ns;
};

template <bool NT>
__device__ __forceinline__ void st(double* p, dvec2 v)
{
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p));
  else *reinterpret_cast<dvec2*>(p) = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) pers(const Args a)
{
  __shared__ double th[128][2];
  for (int i = threadIdx.x; i < a.ns * 2; i += 256) th[i >> 1][i & 1] = a.theta[(a.s0 + (i >> 1)) * 2 + (i & 1)];
  __syncthreads();
  const long n2 = a.nnz >> 1;
  for (long k = long(blockIdx.x) * 256 + threadIdx.x; k < n2; k += long(gridDim.x) * 256) {
    const dvec2 x = reinterpret_cast<const dvec2*>(a.v0)[k];
    const dvec2 y = reinterpret_cast<const dvec2*>(a.v1)[k];
    for (int s = 0; s < a.ns; ++s) {
      const dvec2 r = th[s][0] * x + th[s][1] * y;
      st<NT>(a.out + (a.s0 + s) * a.stride + 2 * k, r);
    }
  }
}

template <bool NT>
__global__ void __launch_bounds__(256) nonp(const Args a)
{
  const long k = long(blockIdx.x) * 256 + threadIdx.x;
  if (k >= (a.nnz >> 1)) return;
  const dvec2 x = reinterpret_cast<const dvec2*>(a.v0)[k];
  const dvec2 y = reinterpret_cast<const dvec2*>(a.v1)[k];
  for (int s = 0; s < a.ns; ++s) {
    const double t0 = a.theta[(a.s0 + s) * 2], t1 = a.theta[(a.s0 + s) * 2 + 1];
    st<NT>(a.out + (a.s0 + s) * a.stride + 2 * k, t0 * x + t1 * y);
  }
}

// workgroup id -> (block, sample, chunk): chunk fastest, then sample, then block; B = CPB chunks of 512 doubles
template <bool NT, int CPB>
__global__ void __launch_bounds__(256) blocked(const Args a)
{
  const long w = blockIdx.x;
  const long per_block = long(CPB) * 128;
  const long blk = w / per_block, rem = w - blk * per_block;
  const int s = int(rem / CPB);
  const long c = blk * CPB + (rem - long(s) * CPB);
  const long k = c * 256 + threadIdx.x;
  if (k >= (a.nnz >> 1)) return;
  const dvec2 x = reinterpret_cast<const dvec2*>(a.v0)[k];
  const dvec2 y = reinterpret_cast<const dvec2*>(a.v1)[k];
  const double t0 = a.theta[s * 2], t1 = a.theta[s * 2 + 1];
  st<NT>(a.out + s * a.stride + 2 * k, t0 * x + t1 * y);
}

int main()
{
  const long nnz = 75460608, S = 128;
  double *v0, *v1, *out, *theta;
  (void)hipMalloc(&v0, nnz * 8); (void)hipMalloc(&v1, nnz * 8);
  (void)hipMalloc(&out, S * nnz * 8); (void)hipMalloc(&theta, S * 2 * 8);
  std::vector<double> th(S * 2), hv(nnz);
  for (long i = 0; i < S * 2; ++i) th[i] = 0.1 + 0.007 * double(i);
  for (long i = 0; i < nnz; ++i) hv[i] = 1.0 + 1e-9 * double(i % 977);
  (void)hipMemcpy(theta, th.data(), S * 2 * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(v0, hv.data(), nnz * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(v1, hv.data(), nnz * 8, hipMemcpyHostToDevice);
  Args a{v0, v1, out, theta, nnz, nnz, 0, 32};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double wr = double(S) * nnz * 8;
    printf("%-36s %8.3f ms  %6.2f TB/s written\n", name, best, wr / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  const long n2 = nnz / 2;
  for (int pass = 0; pass < 2; ++pass) {
    time("pers32 nt (production)", [&] { for (int s0 = 0; s0 < S; s0 += 32) { Args b = a; b.s0 = s0; b.ns = 32; hipLaunchKernelGGL((pers<true>), dim3(4096), dim3(256), 0, 0, b); } });
    time("pers32 plain", [&] { for (int s0 = 0; s0 < S; s0 += 32) { Args b = a; b.s0 = s0; b.ns = 32; hipLaunchKernelGGL((pers<false>), dim3(4096), dim3(256), 0, 0, b); } });
    time("pers128 nt", [&] { Args b = a; b.s0 = 0; b.ns = 128; hipLaunchKernelGGL((pers<true>), dim3(4096), dim3(256), 0, 0, b); });
    time("pers128 plain", [&] { Args b = a; b.s0 = 0; b.ns = 128; hipLaunchKernelGGL((pers<false>), dim3(4096), dim3(256), 0, 0, b); });
    time("pers128 nt grid 2048", [&] { Args b = a; b.s0 = 0; b.ns = 128; hipLaunchKernelGGL((pers<true>), dim3(2048), dim3(256), 0, 0, b); });
    time("pers128 nt grid 8192", [&] { Args b = a; b.s0 = 0; b.ns = 128; hipLaunchKernelGGL((pers<true>), dim3(8192), dim3(256), 0, 0, b); });
    time("nonp32 nt", [&] { for (int s0 = 0; s0 < S; s0 += 32) { Args b = a; b.s0 = s0; b.ns = 32; hipLaunchKernelGGL((nonp<true>), dim3((n2 + 255) / 256), dim3(256), 0, 0, b); } });
    time("nonp32 plain", [&] { for (int s0 = 0; s0 < S; s0 += 32) { Args b = a; b.s0 = s0; b.ns = 32; hipLaunchKernelGGL((nonp<false>), dim3((n2 + 255) / 256), dim3(256), 0, 0, b); } });
    time("nonp8 plain", [&] { for (int s0 = 0; s0 < S; s0 += 8) { Args b = a; b.s0 = s0; b.ns = 8; hipLaunchKernelGGL((nonp<false>), dim3((n2 + 255) / 256), dim3(256), 0, 0, b); } });
    const long chunks = (n2 + 255) / 256;
    time("blocked 2 MB plain", [&] { constexpr int C = 512; hipLaunchKernelGGL((blocked<false, C>), dim3(((chunks + C - 1) / C) * C * 128), dim3(256), 0, 0, a); });
    time("blocked 8 MB plain", [&] { constexpr int C = 2048; hipLaunchKernelGGL((blocked<false, C>), dim3(((chunks + C - 1) / C) * C * 128), dim3(256), 0, 0, a); });
    time("blocked 32 MB plain", [&] { constexpr int C = 8192; hipLaunchKernelGGL((blocked<false, C>), dim3(((chunks + C - 1) / C) * C * 128), dim3(256), 0, 0, a); });
    time("blocked 8 MB nt", [&] { constexpr int C = 2048; hipLaunchKernelGGL((blocked<true, C>), dim3(((chunks + C - 1) / C) * C * 128), dim3(256), 0, 0, a); });
  }
  std::vector<double> o(4);
  (void)hipMemcpy(o.data(), out + 77 * nnz + 1000, 32, hipMemcpyDeviceToHost);
  printf("check %.12f (expect %.12f)\n", o[0], (th[154] + th[155]) * hv[1000]);
  return 0;
}
