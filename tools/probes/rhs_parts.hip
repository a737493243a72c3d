// Instruction cost of the pieces of one RHS evaluation (diagnostic probe, not
// the product): includes the kernel source and launches one kernel per piece
// over N C3-like points; run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace -- ./rhs_parts
// and divide by SQ_WAVES (tools/valu_parts.py --summarize).  "base" only loads
// the inputs and stores one value: subtract it from the others.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math
//         -I include -I rossby-wave-ray-tracing_amd/csrc -o /tmp/rhs_parts tools/probes/rhs_parts.hip
#include "rwrt.hip"

#include <vector>
#include <random>

using namespace rwrt;

struct In {
  const double *lon, *lat, *k, *l, *amp;
};

__global__ void p_base(In in, int64_t n, double* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in.lon[i] + in.lat[i] + in.k[i] + in.l[i] + in.amp[i];
}
__global__ void p_trig(In in, int64_t n, double* out) {
  nm_stage<NM_SINCOS | NM_TAN>();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c, t;
  const auto pre = np_math::nm_sincostan_begin(in.lat[i]);
  np_math::nm_sincostan_end(in.lat[i], pre, s, c, t);
  out[i] = s + c + t + in.lon[i] + in.k[i] + in.l[i] + in.amp[i];
}
__global__ void p_corners(Field F, In in, int64_t n, double* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Corners k = corners(F, py_mod_2pi(in.lon[i]), in.lat[i]);
  out[i] = k.wa + k.wb + k.wc + k.wd + (double)(k.oa ^ k.ob ^ k.oc ^ k.od ^ k.key_x ^ k.key_y) + in.k[i] +
           in.l[i] + in.amp[i];
}
__global__ void p_interp(Field F, In in, int64_t n, double* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double g[11];
  interp11(F, py_mod_2pi(in.lon[i]), in.lat[i], g);
  double s = in.k[i] + in.l[i] + in.amp[i];
  for (int q = 0; q < 11; ++q) s += g[q];
  out[i] = s;
}
__global__ void p_kap(In in, int64_t n, double* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  DivGuard G;
  const KapTermsR w = kap_terms_r(in.k[i], in.l[i], G);
  out[i] = w.kap + w.kap1 + w.kk + w.denom + w.rkk + w.rk1 + w.rden + (G.ok() ? 1.0 : 0.0) + in.lon[i] +
           in.lat[i] + in.amp[i];
}
__global__ void p_tail(Field F, In in, int64_t n, double* out) {
  nm_stage<NM_SINCOS | NM_TAN>();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  // inputs the tail sees, from cheap stand-ins (their cost is in the other probes)
  const double lat = in.lat[i];
  double g[11];
  for (int q = 0; q < 11; ++q) g[q] = in.lon[i] * (q + 1) * 1e-5 + 1e-6;
  const double s = lat, c = 1.0 - 0.5 * lat * lat, tn = lat;
  DivGuard G;
  const KapTermsR kw = kap_terms_r(in.k[i], in.l[i], G);
  const Merc M = merc_factors(lat, c, s);
  double dy[5], ug, vg;
  asm volatile(";@TAIL_BEGIN");
  if (!rhs_tail_fast(g, M, s, c, tn, in.k[i], kw, G, in.amp[i], dy, ug, vg)) {
    asm volatile("");
    rhs_tail_ieee(g, M, s, c, tn, in.k[i], in.l[i], in.amp[i], dy, ug, vg);
  }
  asm volatile(";@TAIL_END");
  out[i] = dy[0] + dy[1] + dy[2] + dy[3] + dy[4] + ug + vg;
}
__global__ void p_rhs(Field F, In in, int64_t n, double* out) {
  nm_stage<NM_SINCOS | NM_TAN>();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double y[5] = {in.lon[i], in.lat[i], in.k[i], in.l[i], in.amp[i]}, dy[5];
  ray_rhs(StaticBG{F}, 0.0, y, dy);
  out[i] = dy[0] + dy[1] + dy[2] + dy[3] + dy[4];
}

int main() {
  const int64_t n = 1 << 22;
  const int W = 145, H = 73;
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> P((size_t)W * H * kNF), lon(n), lat(n), k(n), l(n), amp(n);
  for (auto& v : P) v = (U(rng) - 0.5) * 1e-4;
  for (int64_t i = 0; i < n; ++i) {
    lon[i] = U(rng) * 6.28;
    lat[i] = (U(rng) - 0.5) * 2.6;
    k[i] = 1.0 + 9.0 * U(rng);
    l[i] = (U(rng) - 0.5) * 20.0;
    amp[i] = 1.0 + U(rng);
  }
  double *dP, *d[5], *dout;
  hipMalloc(&dP, P.size() * 8);
  hipMemcpy(dP, P.data(), P.size() * 8, hipMemcpyHostToDevice);
  std::vector<double>* src[5] = {&lon, &lat, &k, &l, &amp};
  for (int j = 0; j < 5; ++j) {
    hipMalloc(&d[j], n * 8);
    hipMemcpy(d[j], src[j]->data(), n * 8, hipMemcpyHostToDevice);
  }
  hipMalloc(&dout, n * 8);
  Field F{dP, W, H, 0.0, 2.5 * kPi / 180.0, -kHalfPi, 2.5 * kPi / 180.0};
  In in{d[0], d[1], d[2], d[3], d[4]};
  const dim3 g((unsigned)(n / 256)), b(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(p_base, g, b, 0, 0, in, n, dout);
    hipLaunchKernelGGL(p_trig, g, b, 0, 0, in, n, dout);
    hipLaunchKernelGGL(p_corners, g, b, 0, 0, F, in, n, dout);
    hipLaunchKernelGGL(p_interp, g, b, 0, 0, F, in, n, dout);
    hipLaunchKernelGGL(p_kap, g, b, 0, 0, in, n, dout);
    hipLaunchKernelGGL(p_tail, g, b, 0, 0, F, in, n, dout);
    hipLaunchKernelGGL(p_rhs, g, b, 0, 0, F, in, n, dout);
  }
  hipDeviceSynchronize();
  printf("rhs_parts done\n");
  return 0;
}
