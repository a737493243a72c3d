// FETCH_SIZE calibration for the C5 access pattern (VERDICT r1
// item 7): known request bytes, read under rocprofv3 --pmc FETCH_SIZE.
//   stream   : 16 B per lane, coalesced, 1 GiB        (the guide's x2 rule)
//   gather192: per lane two random 192-B spans (a lookup's corner pairs
//              (x0,y0)(x0,y1) and (x1,y0)(x1,y1) of 96-B records), 12 x 16-B
//              loads, from a 2 GiB array (far beyond the 256 MiB MALL)
//   gather96 : per lane four random 96-B records (6 x 16-B loads each)
// Prints the requested bytes of each dispatch; the ratio to FETCH_SIZE is the
// calibration factor of that pattern.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/fetch_probe tools/probes/fetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void stream(const double2* __restrict__ src, int64_t n, double* out) {
  double acc = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = src[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.0) out[0] = acc;
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// nrec records of 96 B in src; each lane: `per` random spans of `span` records
template <int SPAN>
__global__ void gather(const double* __restrict__ src, int64_t nrec, int64_t nlanes, int per, double* out) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= nlanes) return;
  double acc = 0.0;
  for (int k = 0; k < per; ++k) {
    const int64_t r = (int64_t)(mix((uint64_t)t * 8 + k) % (uint64_t)(nrec - SPAN));
    const double2* p = reinterpret_cast<const double2*>(src + r * 12);
#pragma unroll
    for (int c = 0; c < 6 * SPAN; ++c) {
      const double2 v = p[c];
      acc += v.x + v.y;
    }
  }
  if (acc == 12345.0) out[0] = acc;
}

int main() {
  const int64_t bytes = 2ll << 30;
  double* src;
  double* out;
  if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(src, 0, bytes) != hipSuccess) return 1;
  const int64_t nrec = bytes / 96;
  const int64_t n16 = (1ll << 30) / 16;
  stream<<<4096, 256>>>(reinterpret_cast<const double2*>(src), n16, out);
  printf("stream:    requested %lld B\n", (long long)(n16 * 16));
  const int64_t lanes = 1 << 20;
  gather<2><<<lanes / 256, 256>>>(src, nrec, lanes, 2, out);
  printf("gather192: requested %lld B (%lld spans of 192 B)\n", (long long)(lanes * 2 * 192), (long long)(lanes * 2));
  gather<1><<<lanes / 256, 256>>>(src, nrec, lanes, 4, out);
  printf("gather96:  requested %lld B (%lld records of 96 B)\n", (long long)(lanes * 4 * 96), (long long)(lanes * 4));
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return 0;
}
