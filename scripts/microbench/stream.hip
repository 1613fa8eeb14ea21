// HBM calibration kernels: 16-byte/lane streaming write (plain / nontemporal), read (sum), copy.
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <cstdio>
#include <vector>
#include <algorithm>
typedef double dvec2 __attribute__((ext_vector_type(2)));
__global__ void wr(dvec2* p, long n, int nt) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    dvec2 v = {(double)i, 1.0};
    if (nt) __builtin_nontemporal_store(v, p + i); else p[i] = v;
  }
}
__global__ void rd(const dvec2* p, long n, double* out) {
  double s = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) { dvec2 v = p[i]; s += v.x + v.y; }
  if (s == 1.2345) *out = s;
}
__global__ void rd8(const double* p, long n, double* out) {
  double s = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += p[i];
  if (s == 1.2345) *out = s;
}
__global__ void wr8(double* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = (double)i;
}
__global__ void cp(const dvec2* a, dvec2* b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) __builtin_nontemporal_store(a[i], b + i);
}
int main() {
  const long bytes = 1200L << 20, n = bytes / 16;
  dvec2 *a, *b; double* o;
  hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&o, 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int grid : {2048, 8192, 32768}) {
    for (int which = 0; which < 6; ++which) {
      std::vector<float> ts;
      for (int r = 0; r < 8; ++r) {
        hipEventRecord(e0);
        if (which == 0) wr<<<grid, 256>>>(a, n, 0);
        if (which == 1) wr<<<grid, 256>>>(a, n, 1);
        if (which == 2) rd<<<grid, 256>>>(a, n, o);
        if (which == 3) cp<<<grid, 256>>>(a, b, n / 2);
        if (which == 4) rd8<<<grid, 256>>>((const double*)a, 2 * n, o);
        if (which == 5) wr8<<<grid, 256>>>((double*)a, 2 * n);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const char* nm[] = {"write", "write_nt", "read", "copy(0.6+0.6GB)", "read_8B_lane", "write_8B_lane"};
      printf("grid %6d %-16s median %.4f ms  %.0f GB/s\n", grid, nm[which], ts[4], bytes / (ts[4] * 1e-3) / 1e9);
    }
  }
  return 0;
}
