// Dependent-latency probe for one lone wave on gfx950 (MI355X): cycles per
// operation of a dependent chain (s_memtime around N chained operations).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/lat_probe tools/probes/lat_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 4096
__global__ void probe(double* out, long long* cyc, double a, double b) {
  double x = a + threadIdx.x * 1e-9, y = b;
  __shared__ double lds[256];
  lds[threadIdx.x] = x;
  __syncthreads();
  long long t0, t1;
  // 0: dependent v_fma_f64
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) x = __builtin_fma(x, a, b);
  asm volatile("" : "+v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  // 1: dependent v_add_f64
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) x = x + b;
  asm volatile("" : "+v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[1] = t1 - t0;
  // 2: independent v_fma_f64 x4 chains (issue rate)
  double x1 = x + 1, x2 = x + 2, x3 = x + 3;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    x = __builtin_fma(x, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
  }
  asm volatile("" : "+v"(x), "+v"(x1), "+v"(x2), "+v"(x3));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[2] = t1 - t0;
  // 3: dependent IEEE division
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N / 16; ++i) y = a / (y + 1.5);
  asm volatile("" : "+v"(y));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[3] = t1 - t0;
  // 4: dependent v_rcp_f64
  double r = y;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N / 4; ++i) r = __builtin_amdgcn_rcp(r);
  asm volatile("" : "+v"(r));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[4] = t1 - t0;
  // 5: dependent LDS read (pointer chase through a value)
  int idx = threadIdx.x;
  int* li = (int*)lds;
  li[threadIdx.x] = (threadIdx.x + 1) & 255;
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N / 16; ++i) idx = li[idx];
  asm volatile("" : "+v"(idx));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[5] = t1 - t0;
  // 6: dependent v_mul_f64
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) x = x * a;
  asm volatile("" : "+v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[6] = t1 - t0;
  // 7: dependent v_cndmask chain on f64 compares
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N / 4; ++i) x = (x > b) ? x * 0.5 : x + a;
  asm volatile("" : "+v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[7] = t1 - t0;
  // 8: s_memtime back to back
  t0 = __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[8] = t1 - t0;
  out[threadIdx.x] = x + y + r + idx + x1 + x2 + x3;
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) const void* global_void_ptr;
// LDS-DMA issue and completion cost: 24 global_load_lds_dwordx4 (a cell-cache
// refill) with `active` lanes of the wave, from an L2-resident 1 MB table
__global__ void dma_probe(const double* __restrict__ src, long long* cyc, int active, int reps) {
  __shared__ __attribute__((aligned(16))) char buf[24 * 1024];
  const int lane = threadIdx.x & 63;
  long long t_issue = 0, t_wait = 0;
  if (lane < active) {
    for (int r = 0; r < reps; ++r) {
      const double* p = src + ((r * 977 + lane * 131) % 8192) * 12;
      long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
      for (int c = 0; c < 24; ++c)
        __builtin_amdgcn_global_load_lds((global_void_ptr)(p + (c / 6) * 12 * 73 + (c % 6) * 2),
                                         (lds_void_ptr)(buf + c * 1024), 16, 0, 0);
      long long t1 = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      long long t2 = __builtin_amdgcn_s_memtime();
      t_issue += t1 - t0;
      t_wait += t2 - t1;
    }
  }
  if (threadIdx.x == 0) {
    cyc[0] = t_issue;
    cyc[1] = t_wait;
  }
}
// the same 24 chunks as 24 plain 16-B global loads into registers
__global__ void load_probe(const double* __restrict__ src, long long* cyc, double* out, int active, int reps) {
  const int lane = threadIdx.x & 63;
  long long t_all = 0;
  double acc = 0.0;
  if (lane < active) {
    for (int r = 0; r < reps; ++r) {
      const double* p = src + ((r * 977 + lane * 131) % 8192) * 12;
      long long t0 = __builtin_amdgcn_s_memtime();
      double2 v[24];
#pragma unroll
      for (int c = 0; c < 24; ++c) v[c] = *(const double2*)(p + (c / 6) * 12 * 73 + (c % 6) * 2);
#pragma unroll
      for (int c = 0; c < 24; ++c) acc += v[c].x + v[c].y;
      asm volatile("" : "+v"(acc));
      long long t1 = __builtin_amdgcn_s_memtime();
      t_all += t1 - t0;
    }
  }
  if (threadIdx.x == 0) cyc[2] = t_all;
  out[threadIdx.x] = acc;
}

int main() {
  double* out; long long* cyc;
  hipMalloc(&out, 256 * sizeof(double));
  hipMalloc(&cyc, 16 * sizeof(long long));
  long long h[16];
  const char* names[] = {"fma f64 dep", "add f64 dep", "fma f64 4 indep chains (per fma)", "IEEE div f64 dep",
                         "rcp f64 dep", "ds_read_b32 dep", "mul f64 dep", "cmp+cndmask+mul/add dep", "s_memtime pair"};
  const double per[] = {N, N, 4.0 * N, N / 16, N / 4, N / 16, N, N / 4, 1};
  for (int threads : {64, 256}) {
    for (int rep = 0; rep < 2; ++rep) {
      probe<<<1, threads>>>(out, cyc, 0.999999, 1e-7);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("block of %d threads (s_memtime ticks; memtime = shader clock?)\n", threads);
    for (int k = 0; k < 9; ++k) printf("  %-36s %8.2f per op\n", names[k], h[k] / per[k]);
  }
  double* src;
  hipMalloc(&src, 8192 * 12 * 8 * 4);
  hipMemset(src, 0, 8192 * 12 * 8 * 4);
  for (int active : {1, 8, 64}) {
    const int reps = 200;
    for (int rep = 0; rep < 2; ++rep) {
      dma_probe<<<1, 64>>>(src, cyc, active, reps);
      load_probe<<<1, 64>>>(src, cyc, out, active, reps);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("refill of 24 x 16 B with %2d active lanes: LDS-DMA issue %7.1f + wait %7.1f cyc; 24 plain loads + use %7.1f cyc\n",
           active, (double)h[0] / reps, (double)h[1] / reps, (double)h[2] / reps);
  }
  return 0;
}
