// Write-stream microbenchmark, part 3: the C2 store phase with cooperative workgroups.
// wstream2 showed that dense concurrent write windows stream faster (a fill whose 64-lane workgroups write
// adjacent 2 KB chunks, XCD eighths: 6.65 TB/s) than waves that each stream their own 18 KB tile (the
// concurrent addresses of an XCD's waves are 18 KB apart: 6.0-6.2 TB/s).  Here a workgroup of NW waves owns
// NW adjacent tiles (one contiguous CSR range) and, after a barrier, streams the joint image with instruction
// k of wave w writing KB (k NW + w): the workgroup's concurrent writes form one NW KB window.  The region is
// offset by 80 B (16-B but not 128-B aligned), as real tile bases are.
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result wstream3.hip -o wstream3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 36, IMG = 64 * RB, SKEW = 10;

template <int NW, int AUX>
__global__ void __launch_bounds__(64 * NW) coop(double* out, long ntiles)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long ng = ntiles / NW;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  for (int j = 0; j < RB; ++j) lds[wv * IMG + lane * RB + j] = j;
  constexpr int LEN = NW * IMG, ST = (LEN / 2 + 64 * NW - 1) / (64 * NW);
  for (long g = (ng * x) / 8 + w; g < (ng * (x + 1)) / 8; g += gx) {
    __syncthreads();   // image complete (models compute -> LDS of every wave)
    __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(out + SKEW + g * LEN, (short)0, LEN * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int idx = 2 * ((k * NW + wv) * 64 + lane);
      const dvec2 v = *reinterpret_cast<const dvec2*>(lds + (idx < LEN ? idx : 0));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, AUX);
    }
  }
}

// baseline: each wave streams its own tile (production store phase), same skew
template <int AUX>
__global__ void __launch_bounds__(64, 1) own(double* out, long ntiles)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  constexpr int ST = (IMG / 2 + 63) / 64;
  for (long t = (ntiles * x) / 8 + w; t < (ntiles * (x + 1)) / 8; t += gx) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + SKEW + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int idx = 2 * (lane + 64 * k);
      const dvec2 v = *reinterpret_cast<const dvec2*>(lds + (idx < IMG ? idx : 0));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, AUX);
    }
  }
}

int main()
{
  const long ntiles = 64000, n = ntiles * IMG + 64;
  double* out;
  (void)hipMalloc(&out, n * 8);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const double bytes = double(ntiles) * IMG * 8;
  auto time = [&](const char* name, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 20;
      best = ms < best ? ms : best;
    }
    printf("%-40s %8.4f ms  %6.2f TB/s\n", name, best, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  char nm[96];
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&coop<8, 2>), hipFuncAttributeMaxDynamicSharedMemorySize, 8 * IMG * 8);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&coop<8, 0>), hipFuncAttributeMaxDynamicSharedMemorySize, 8 * IMG * 8);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&coop<4, 2>), hipFuncAttributeMaxDynamicSharedMemorySize, 4 * IMG * 8);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&coop<4, 0>), hipFuncAttributeMaxDynamicSharedMemorySize, 4 * IMG * 8);
#define COOP(NW, AUX, WPC)                                                                                   \
  snprintf(nm, sizeof nm, "coop NW=%d aux=%d waves/CU=%d", NW, AUX, WPC);                                 \
  time(nm, [&] { hipLaunchKernelGGL((coop<NW, AUX>), dim3(cus * (WPC) / (NW)), dim3(64 * NW),              \
                                    size_t(NW) * IMG * 8, 0, out, ntiles); })
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d (%.3f GB, %d CUs)\n", pass, bytes / 1e9, cus);
    for (int wpc : {2, 4, 8}) {
      snprintf(nm, sizeof nm, "own nt waves/CU=%d", wpc);
      time(nm, [&] { hipLaunchKernelGGL((own<2>), dim3(cus * wpc), dim3(64), 0, 0, out, ntiles); });
      snprintf(nm, sizeof nm, "own plain waves/CU=%d", wpc);
      time(nm, [&] { hipLaunchKernelGGL((own<0>), dim3(cus * wpc), dim3(64), 0, 0, out, ntiles); });
    }
    COOP(2, 2, 4); COOP(2, 0, 4); COOP(2, 2, 8); COOP(2, 0, 8);
    COOP(4, 2, 4); COOP(4, 0, 4); COOP(4, 2, 8); COOP(4, 0, 8);
    COOP(8, 2, 8); COOP(8, 0, 8);
  }
  return 0;
}
