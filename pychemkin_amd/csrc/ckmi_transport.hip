// ckmi_transport.hip -- pure-species and mixture viscosity and thermal conductivity on gfx950
// (SURVEY.md §8(f) rank 4).
//
// The reference reads a Chemkin transport file at preprocess (chemistry.py:636-687, itran = 1) and
// its closed library evaluates viscosities on demand: KINGetViscosity (species, mixture.py:1860-1883)
// and KINGetMixtureViscosity (mixture.py:1943-1977), the latter on every saved point of a reactor
// solution in the reference's own tests (CONV.py:176-190).  Restated method (TRANFIT / TRANLIB):
//
//   fit (host, once per mechanism):
//     eta_k(T) = 5/16 sqrt(pi m_k kB T) / (pi sigma_k^2 Omega22*(T / eps_k, delta*_k)),
//     Omega22* = 1.16145 T*^-0.14874 + 0.52487 e^(-0.7732 T*) + 2.16178 e^(-2.43787 T*) + 0.2 delta*^2 / T*
//     (Neufeld-Janzen-Aziz correlation of the Lennard-Jones table, Brokaw's polar term), and
//     ln eta_k = sum_n a_kn (ln T)^n, n < 4, least squares (Householder QR) on 50 temperatures
//     equally spaced in [tlow, thigh];
//   evaluate (device, one state per lane):
//     eta_k = exp(poly), eta = sum_k X_k eta_k / sum_j X_j Phi_kj (Wilke),
//     Phi_kj = A_kj (1 + s_k B_kj / s_j)^2, s = sqrt(eta), A_kj = (1 + W_k / W_j)^-1/2 / sqrt 8,
//     B_kj = (W_j / W_k)^1/4 (A, B precomputed per mechanism, read by wave-uniform scalar loads).
//
// Layout: SoA like the ROP kernel (Y[KK][n], lane = state).  Per lane the species vectors X_j and
// 1 / s_j live in a per-thread LDS column ([KK][block] doubles, conflict-free), so the KK^2 Wilke
// double loop reads its lane's vectors from LDS and the (k, j) table entries from the scalar cache.
// Bound: FP64 VALU (KK^2 x 6 FLOP per state); HBM traffic is (KK + 2) x 8 B per state.
// Conductivity (KINGetConductivity / KINGetMixtureConductivity, mixture.py:1885-1909,1979-2013):
// lambda_k from the ln-T cubic of ckmi_conductivity_fit, mixed by lambda = (sum X lambda + 1 / sum X / lambda) / 2.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "ckmi_internal.hpp"

struct ckmi_transport {
  int device = 0;
  int KK = 0;
  double* fits = nullptr;  // device [KK][4]
  double* A = nullptr;     // device [KK][KK]
  double* B = nullptr;     // device [KK][KK]
  double* cfits = nullptr; // device [KK][4] conductivity fits (ckmi_transport_set_conductivity), else NULL
  const double* wt = nullptr;  // the mechanism's device weights
  std::vector<double> fits_host;
  std::vector<double> cfits_host;
};

namespace {

constexpr double KB = 1.380649e-16;       // erg / K
constexpr double NA = 6.02214076e23;
constexpr double DEBYE = 1e-18;           // esu cm
constexpr double ANGSTROM = 1e-8;         // cm
constexpr int FIT_NPTS = 50;
constexpr int FIT_ORDER = 4;

int fail(int code, const std::string& msg) { return ckmi::set_error(code, msg); }

double omega22(double tstar, double dstar) {
  return 1.16145 * std::pow(tstar, -0.14874) + 0.52487 * std::exp(-0.77320 * tstar) +
         2.16178 * std::exp(-2.43787 * tstar) + 0.2 * dstar * dstar / tstar;
}

// least squares min |V c - y| for the FIT_NPTS x FIT_ORDER Vandermonde matrix V by Householder QR
void lsq_qr(double (*V)[FIT_ORDER], double* y, double* c) {
  constexpr int m = FIT_NPTS, n = FIT_ORDER;
  for (int j = 0; j < n; ++j) {
    double nrm = 0.0;
    for (int i = j; i < m; ++i) nrm += V[i][j] * V[i][j];
    nrm = std::sqrt(nrm);
    const double alpha = V[j][j] > 0 ? -nrm : nrm;
    double v[m];
    for (int i = 0; i < m; ++i) v[i] = i < j ? 0.0 : V[i][j];
    v[j] -= alpha;
    double vv = 0.0;
    for (int i = j; i < m; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    for (int k = j; k < n; ++k) {
      double s = 0.0;
      for (int i = j; i < m; ++i) s += v[i] * V[i][k];
      s = 2.0 * s / vv;
      for (int i = j; i < m; ++i) V[i][k] -= s * v[i];
    }
    double s = 0.0;
    for (int i = j; i < m; ++i) s += v[i] * y[i];
    s = 2.0 * s / vv;
    for (int i = j; i < m; ++i) y[i] -= s * v[i];
  }
  for (int j = n - 1; j >= 0; --j) {
    double s = y[j];
    for (int k = j + 1; k < n; ++k) s -= V[j][k] * c[k];
    c[j] = s / V[j][j];
  }
}

__global__ void species_viscosity_kernel(int KK, int n, const double* __restrict__ fits, const double* __restrict__ T,
                                         double* __restrict__ visc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = log(T[i]);
  for (int k = 0; k < KK; ++k) {
    const double* a = fits + 4 * k;
    visc[(size_t)k * n + i] = exp(fma(x, fma(x, fma(x, a[3], a[2]), a[1]), a[0]));
  }
}

// one state per lane; dynamic LDS: X [KK][blockDim] then 1/sqrt(eta) [KK][blockDim]
__global__ void mixture_viscosity_kernel(int KK, int n, const double* __restrict__ fits, const double* __restrict__ A,
                                         const double* __restrict__ B, const double* __restrict__ wt,
                                         const double* __restrict__ T, const double* __restrict__ Y,
                                         double* __restrict__ visc) {
  extern __shared__ double tv_lds[];
  const int bs = blockDim.x, t = threadIdx.x;
  const int i = blockIdx.x * bs + t;
  const bool live = i < n;
  const int ii = live ? i : 0;
  double* Xs = tv_lds + t;            // Xs[k * bs]
  double* Rs = tv_lds + KK * bs + t;  // Rs[k * bs] = 1 / sqrt(eta_k)
  const double x = log(T[ii]);
  // x_k = Y_k / W_k: the Wilke ratio is homogeneous of degree 0 in X, so the normalisation
  // sum_j x_j cancels between each numerator and its denominator
  // negative trace mass fractions (integrator output) count as 0, as in the engine's wall-heat path
  // (ckmi_reactor.hpp engine_hA)
  for (int k = 0; k < KK; ++k) {
    const double xk = fmax(Y[(size_t)k * n + ii], 0.0) / wt[k];
    Xs[k * bs] = xk;
    const double* a = fits + 4 * k;
    Rs[k * bs] = exp(-0.5 * fma(x, fma(x, fma(x, a[3], a[2]), a[1]), a[0]));
  }
  double mix = 0.0;
  for (int k = 0; k < KK; ++k) {
    const double xk = Xs[k * bs];
    if (xk == 0.0) continue;  // X_k eta_k / den_k = 0 (den_k >= X_k A_kk 4 > 0 otherwise)
    const double rk = Rs[k * bs];
    const double sk = 1.0 / rk;
    const double* Ak = A + (size_t)k * KK;
    const double* Bk = B + (size_t)k * KK;
    double den = 0.0;
    for (int j = 0; j < KK; ++j) {
      const double f = fma(sk * Rs[j * bs], Bk[j], 1.0);
      den = fma(Xs[j * bs] * Ak[j], f * f, den);
    }
    mix += xk * (sk * sk) / den;
  }
  if (live) visc[i] = mix;
}

// one state per lane: X_k = (Y_k^+ / W_k) / sum_j Y_j^+ / W_j (Y^+ = max(Y, 0)), lambda_k = exp(poly_k(ln T)),
// lambda = (sum_k X_k lambda_k + 1 / sum_k X_k / lambda_k) / 2 (Chemkin's mixture-averaged rule, the
// form the engine's wall heat transfer evaluates in ckmi_reactor.hpp).  Species with X_k = 0 add
// nothing to either sum.  KK x (2 FLOP + exp) per state: FP64 VALU / transcendental bound.
__global__ void mixture_conductivity_kernel(int KK, int n, const double* __restrict__ cfits,
                                            const double* __restrict__ wt, const double* __restrict__ T,
                                            const double* __restrict__ Y, double* __restrict__ cond) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = log(T[i]);
  double sx = 0.0, sxl = 0.0, sxr = 0.0;
  for (int k = 0; k < KK; ++k) {
    const double xk = fmax(Y[(size_t)k * n + i], 0.0) / wt[k];  // negative traces count as 0 (engine_hA)
    if (xk == 0.0) continue;
    const double* a = cfits + 4 * k;
    const double lk = exp(fma(x, fma(x, fma(x, a[3], a[2]), a[1]), a[0]));
    sx += xk;
    sxl = fma(xk, lk, sxl);
    sxr += xk / lk;
  }
  // with x_k unnormalised: sum X lambda = sxl / sx, 1 / sum X / lambda = sx / sxr
  cond[i] = sx > 0.0 ? 0.5 * (sxl / sx + sx / sxr) : 0.0;
}

}  // namespace

extern "C" {

int ckmi_transport_fit(int32_t KK, const double* wt, const double* params, double tlow, double thigh, double* fits) {
  if (KK <= 0 || !wt || !params || !fits) return fail(CKMI_ERR_ARG, "ckmi_transport_fit: bad argument");
  if (!(tlow > 0.0) || !(thigh > tlow)) return fail(CKMI_ERR_ARG, "ckmi_transport_fit: need 0 < tlow < thigh");
  for (int k = 0; k < KK; ++k) {
    const double* p = params + 6 * k;
    const double eps = p[1], sig = p[2] * ANGSTROM, mu = p[3] * DEBYE;
    if (!(eps > 0.0) || !(sig > 0.0) || !(wt[k] > 0.0))
      return fail(CKMI_ERR_ARG, "ckmi_transport_fit: species " + std::to_string(k) + " needs eps/k > 0, sigma > 0, W > 0");
    const double dstar = 0.5 * mu * mu / (eps * KB * sig * sig * sig);
    const double m = wt[k] / NA;
    double V[FIT_NPTS][FIT_ORDER], y[FIT_NPTS];
    for (int i = 0; i < FIT_NPTS; ++i) {
      const double T = tlow + (thigh - tlow) * i / (FIT_NPTS - 1);
      const double eta = (5.0 / 16.0) * std::sqrt(M_PI * m * KB * T) / (M_PI * sig * sig * omega22(T / eps, dstar));
      const double x = std::log(T);
      V[i][0] = 1.0;
      for (int j = 1; j < FIT_ORDER; ++j) V[i][j] = V[i][j - 1] * x;
      y[i] = std::log(eta);
    }
    lsq_qr(V, y, fits + FIT_ORDER * k);
  }
  return CKMI_OK;
}

int ckmi_conductivity_fit(int32_t KK, const double* wt, const double* params, const double* thermo, double tlow,
                          double thigh, double* fits) {
  // lambda_k = eta_k / W_k (f_tr Cv_tr + f_rot Cv_rot + f_vib Cv_vib) (Warnatz; TRANFIT), rho D_kk / eta_k
  // from the self-diffusion coefficient with Omega11* (Neufeld) + 0.19 delta*^2 / T*, Zrot(T) by Parker's
  // F(T*), Cv_vib = Cv - Cv_tr - Cv_rot from the NASA-7 cp; atoms 15/4 R eta / W; then a cubic in ln T
  if (KK <= 0 || !wt || !params || !thermo || !fits) return fail(CKMI_ERR_ARG, "ckmi_conductivity_fit: bad argument");
  if (!(tlow > 0.0) || !(thigh > tlow)) return fail(CKMI_ERR_ARG, "ckmi_conductivity_fit: need 0 < tlow < thigh");
  const double R = KB * NA;
  auto parker = [](double ts) {
    const double r = 1.0 / ts;
    return 1.0 + 0.5 * std::pow(M_PI, 1.5) * std::sqrt(r) + (0.25 * M_PI * M_PI + 2.0) * r + std::pow(M_PI, 1.5) * r * std::sqrt(r);
  };
  for (int k = 0; k < KK; ++k) {
    const double* p = params + 6 * k;
    const int geo = (int)p[0];
    const double eps = p[1], sig = p[2] * ANGSTROM, mu = p[3] * DEBYE, zrot = p[5];
    if (!(eps > 0.0) || !(sig > 0.0) || !(wt[k] > 0.0))
      return fail(CKMI_ERR_ARG, "ckmi_conductivity_fit: species " + std::to_string(k) + " needs eps/k > 0, sigma > 0, W > 0");
    const double dstar = 0.5 * mu * mu / (eps * KB * sig * sig * sig);
    const double m = wt[k] / NA;
    const double* th = thermo + 17 * k;
    double V[FIT_NPTS][FIT_ORDER], y[FIT_NPTS];
    for (int i = 0; i < FIT_NPTS; ++i) {
      const double T = tlow + (thigh - tlow) * i / (FIT_NPTS - 1);
      const double ts = T / eps;
      const double eta = (5.0 / 16.0) * std::sqrt(M_PI * m * KB * T) / (M_PI * sig * sig * omega22(ts, dstar));
      double lam;
      if (geo == 0) {
        lam = 3.75 * R * eta / wt[k];
      } else {
        const double om11 = 1.06036 * std::pow(ts, -0.15610) + 0.19300 * std::exp(-0.47635 * ts) +
                            1.03587 * std::exp(-1.52996 * ts) + 1.76474 * std::exp(-3.89411 * ts) + 0.19 * dstar * dstar / ts;
        const double kT = KB * T;
        const double rhoD = 3.0 / 16.0 * std::sqrt(2.0 * M_PI * kT * kT * kT / (0.5 * m)) / (M_PI * sig * sig * om11) * m / kT;
        const double x = rhoD / eta;
        const double* a = T > th[1] ? th + 10 : th + 3;
        const double cv = a[0] + T * (a[1] + T * (a[2] + T * (a[3] + T * a[4]))) - 1.0;  // cv / R
        const double cvt = 1.5, cvr = geo == 1 ? 1.0 : 1.5, cvv = cv - cvt - cvr;
        const double Z = zrot * parker(298.0 / eps) / parker(ts);
        const double A = 2.5 - x, Bc = Z + 2.0 / M_PI * (5.0 / 3.0 * cvr + x);
        const double ftr = 2.5 * (1.0 - 2.0 / M_PI * cvr / cvt * A / Bc);
        const double frot = x * (1.0 + 2.0 / M_PI * A / Bc);
        lam = eta / wt[k] * R * (ftr * cvt + frot * cvr + x * cvv);
      }
      const double lx = std::log(T);
      V[i][0] = 1.0;
      for (int j = 1; j < FIT_ORDER; ++j) V[i][j] = V[i][j - 1] * lx;
      y[i] = std::log(lam);
    }
    lsq_qr(V, y, fits + FIT_ORDER * k);
  }
  return CKMI_OK;
}

int ckmi_transport_create(const ckmi_mech* m, const double* fits, ckmi_transport** out) {
  if (!m || !fits || !out) return fail(CKMI_ERR_ARG, "ckmi_transport_create: null argument");
  const int KK = m->KK;
  std::vector<double> W(KK), A((size_t)KK * KK), B((size_t)KK * KK);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != m->device) (void)hipSetDevice(m->device);
  auto* t = new ckmi_transport();
  t->device = m->device;
  t->KK = KK;
  t->wt = m->d.wt;
  t->fits_host.assign(fits, fits + (size_t)FIT_ORDER * KK);
  int rc = CKMI_OK;
  if (hipMemcpy(W.data(), m->d.wt, sizeof(double) * KK, hipMemcpyDeviceToHost) != hipSuccess) {
    rc = fail(CKMI_ERR_HIP, "ckmi_transport_create: reading the mechanism's weights failed");
  } else {
    for (int k = 0; k < KK; ++k)
      for (int j = 0; j < KK; ++j) {
        A[(size_t)k * KK + j] = 1.0 / (std::sqrt(8.0) * std::sqrt(1.0 + W[k] / W[j]));
        B[(size_t)k * KK + j] = std::sqrt(std::sqrt(W[j] / W[k]));
      }
    if (hipMalloc(&t->fits, sizeof(double) * FIT_ORDER * KK) != hipSuccess ||
        hipMalloc(&t->A, sizeof(double) * KK * KK) != hipSuccess || hipMalloc(&t->B, sizeof(double) * KK * KK) != hipSuccess ||
        hipMemcpy(t->fits, fits, sizeof(double) * FIT_ORDER * KK, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(t->A, A.data(), sizeof(double) * KK * KK, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(t->B, B.data(), sizeof(double) * KK * KK, hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(CKMI_ERR_HIP, "ckmi_transport_create: device allocation / upload failed");
  }
  if (prev >= 0 && prev != m->device) (void)hipSetDevice(prev);
  if (rc != CKMI_OK) {
    ckmi_transport_destroy(t);
    return rc;
  }
  *out = t;
  return CKMI_OK;
}

int ckmi_transport_set_conductivity(ckmi_transport* t, const double* cfits) {
  if (!t || !cfits) return fail(CKMI_ERR_ARG, "ckmi_transport_set_conductivity: null argument");
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != t->device) (void)hipSetDevice(t->device);
  int rc = CKMI_OK;
  if (!t->cfits && hipMalloc(&t->cfits, sizeof(double) * FIT_ORDER * t->KK) != hipSuccess)
    rc = fail(CKMI_ERR_HIP, "ckmi_transport_set_conductivity: device allocation failed");
  else if (hipMemcpy(t->cfits, cfits, sizeof(double) * FIT_ORDER * t->KK, hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(CKMI_ERR_HIP, "ckmi_transport_set_conductivity: upload failed");
  else
    t->cfits_host.assign(cfits, cfits + (size_t)FIT_ORDER * t->KK);
  if (prev >= 0 && prev != t->device) (void)hipSetDevice(prev);
  return rc;
}

int ckmi_species_conductivity(const ckmi_transport* t, int32_t n, const double* T, double* cond, void* stream) {
  if (!t || n < 0 || !T || !cond) return fail(CKMI_ERR_ARG, "ckmi_species_conductivity: bad argument");
  if (!t->cfits) return fail(CKMI_ERR_ARG, "ckmi_species_conductivity: no conductivity fits (ckmi_transport_set_conductivity)");
  if (n == 0) return CKMI_OK;
  const int bs = 256;
  // the same ln-T cubic evaluation as the species viscosities, on the conductivity fits
  hipLaunchKernelGGL(species_viscosity_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, (hipStream_t)stream, t->KK, n,
                     t->cfits, T, cond);
  if (hipGetLastError() != hipSuccess) return fail(CKMI_ERR_HIP, "species conductivity launch failed");
  return CKMI_OK;
}

int ckmi_mixture_conductivity(const ckmi_transport* t, int32_t n, const double* T, const double* Y, double* cond,
                              void* stream) {
  if (!t || n < 0 || !T || !Y || !cond) return fail(CKMI_ERR_ARG, "ckmi_mixture_conductivity: bad argument");
  if (!t->cfits) return fail(CKMI_ERR_ARG, "ckmi_mixture_conductivity: no conductivity fits (ckmi_transport_set_conductivity)");
  if (n == 0) return CKMI_OK;
  const int bs = 256;
  hipLaunchKernelGGL(mixture_conductivity_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, (hipStream_t)stream, t->KK, n,
                     t->cfits, t->wt, T, Y, cond);
  if (hipGetLastError() != hipSuccess) return fail(CKMI_ERR_HIP, "mixture_conductivity_kernel launch failed");
  return CKMI_OK;
}

int ckmi_transport_destroy(ckmi_transport* t) {
  if (!t) return CKMI_OK;
  (void)hipFree(t->cfits);
  (void)hipFree(t->fits);
  (void)hipFree(t->A);
  (void)hipFree(t->B);
  delete t;
  return CKMI_OK;
}

int ckmi_transport_fits(const ckmi_transport* t, double* fits) {
  if (!t || !fits) return fail(CKMI_ERR_ARG, "ckmi_transport_fits: null argument");
  std::copy(t->fits_host.begin(), t->fits_host.end(), fits);
  return CKMI_OK;
}

int ckmi_species_viscosity(const ckmi_transport* t, int32_t n, const double* T, double* visc, void* stream) {
  if (!t || n < 0 || !T || !visc) return fail(CKMI_ERR_ARG, "ckmi_species_viscosity: bad argument");
  if (n == 0) return CKMI_OK;
  const int bs = 256;
  hipLaunchKernelGGL(species_viscosity_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, (hipStream_t)stream, t->KK, n,
                     t->fits, T, visc);
  if (hipGetLastError() != hipSuccess) return fail(CKMI_ERR_HIP, "species_viscosity_kernel launch failed");
  return CKMI_OK;
}

int ckmi_mixture_viscosity(const ckmi_transport* t, int32_t n, const double* T, const double* Y, double* visc,
                           void* stream) {
  if (!t || n < 0 || !T || !Y || !visc) return fail(CKMI_ERR_ARG, "ckmi_mixture_viscosity: bad argument");
  if (n == 0) return CKMI_OK;
  // one wave per block up to 150 species (<= 150 KB of LDS), half a wave above
  const int bs = t->KK <= 150 ? 64 : 32;
  const size_t lds = sizeof(double) * 2 * (size_t)t->KK * bs;
  if (lds > 160 * 1024) return fail(CKMI_ERR_UNSUPPORTED, "ckmi_mixture_viscosity: more than 255 species");
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)mixture_viscosity_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return fail(CKMI_ERR_HIP, "ckmi_mixture_viscosity: LDS attribute failed");
  hipLaunchKernelGGL(mixture_viscosity_kernel, dim3((n + bs - 1) / bs), dim3(bs), lds, (hipStream_t)stream, t->KK, n,
                     t->fits, t->A, t->B, t->wt, T, Y, visc);
  if (hipGetLastError() != hipSuccess) return fail(CKMI_ERR_HIP, "mixture_viscosity_kernel launch failed");
  return CKMI_OK;
}

}  // extern "C"
