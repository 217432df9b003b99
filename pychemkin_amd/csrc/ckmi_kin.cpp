// ckmi_kin.cpp -- KIN-compatible C ABI shims (include/ckmi_kin.h) over the batched ckmi engine.
//
// The reference drives one native 0-D reactor per process through a sequence of by-pointer calls
// (batchreactor.py:1149-1159, :1036-1047, :1083-1114): Setup -> SetupBatchInputs -> profile and
// keyword text -> Calculate -> GetIgnitionDelay / GetGasSolnResponse.  This file keeps that global
// state machine on the host (guarded by a mutex: the reference's library is not re-entrant either),
// translates the keyword text into the typed ckmi_reactor_cfg, and runs the reactor as a batch of
// one on the GPU kernels of ckmi.hip / ckmi_big.hip.  Per-state thermo / ROP calls stage their
// state into a small device buffer of the chemistry set and run the batched kernels with n = 1.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "../../include/ckmi_kin.h"

namespace {

constexpr double RU = 1.3806504e-16 * 6.02214179e23;  // erg/mol-K (reference constants.py:37)
constexpr int NAME_LEN = 16;                            // MAX_SPECIES_LENGTH - 1 (chemistry.py:41-43)
constexpr int MAX_ADAP = 20000;                         // adaptive solution points per run

thread_local std::string g_err;
std::recursive_mutex g_mu;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct ChemSet {
  ckmi_mech* mech = nullptr;
  int device = 0, KK = 0, II = 0, MM = 0;
  std::vector<double> wt, awt, thermo;  // thermo [KK][17] for the per-mass conversions
  std::vector<int32_t> ncf;             // [MM][KK] row-major
  std::vector<std::string> names, elements;
  std::vector<std::string> equations;   // reaction strings (KINPreProcess sets; KINGetGasReactionString)
  double* dbuf = nullptr;               // device scratch for single-state calls
  size_t dbuf_n = 0;
  ckmi_transport* tran = nullptr;       // viscosity fits (KINPreProcess with itran = 1)
  double* dtran = nullptr;              // device [KK][8] viscosity + conductivity fits (engine heat transfer)
};
std::vector<ChemSet*> g_sets;  // chemistry set id = index + 1
int g_active = 0;

ChemSet* get_set(const int* id) {
  if (!id || *id < 1 || *id > (int)g_sets.size() || !g_sets[*id - 1]) return nullptr;
  return g_sets[*id - 1];
}

struct Profile {
  std::string key;
  std::vector<double> x, y;
};

// the one configured 0-D reactor (KINAll0D_*), as in the reference's native library
struct Reactor0D {
  int chemset = 0, problem = 0, energy = 0;
  int reactortype = 1;  // 1 batch, 3 plug flow (problem 3 of ckmi_reactor_run: x [cm] is the variable),
                        // 4 HCCI engine (problem 4: V(t) from the crank, eng below)
  double eng[20] = {};  // engine: the CKMI_ENG_* block (KINAll0D_SetupHCCIInputs + engine keywords)
  bool setup = false, inputs = false;
  double t_end = 0, T0 = 0, P0 = 0, V0 = 0, qloss = 0;
  double x0 = 0;        // plug flow: start position [cm] (output positions are x0 + the integration variable)
  std::vector<double> Y0;
  std::vector<std::pair<std::string, std::string>> kw;  // keyword, value text (in order)
  std::vector<Profile> prof;
  // results
  bool done = false;
  double tau = -1.0;
  std::vector<double> t, T, P, V, Y;  // Y [npts][KK]
  ckmi_reactor_cfg cfg{};             // the configuration the last run was integrated with
};
Reactor0D g_r;

std::string upper(std::string s) {
  for (char& c : s) c = (char)std::toupper((unsigned char)c);
  return s;
}
std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

int hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(CKMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return CKMI_OK;
}

int ensure_scratch(ChemSet* s, size_t n) {
  if (s->dbuf_n >= n) return CKMI_OK;
  if (s->dbuf) (void)hipFree(s->dbuf);
  s->dbuf = nullptr;
  s->dbuf_n = 0;
  int rc = hip_ok(hipMalloc((void**)&s->dbuf, n * sizeof(double)), "hipMalloc");
  if (rc == CKMI_OK) s->dbuf_n = n;
  return rc;
}

// cp/R, h/RT, s/R of every species at T on the device (ckmi_species_thermo, n = 1)
int species_thermo(ChemSet* s, double T, std::vector<double>& cpR, std::vector<double>& hRT,
                   std::vector<double>& sR) {
  const int KK = s->KK;
  int rc = ensure_scratch(s, 1 + 3 * (size_t)KK);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, &T, sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  rc = ckmi_species_thermo(s->mech, 1, s->dbuf, s->dbuf + 1, s->dbuf + 1 + KK, s->dbuf + 1 + 2 * KK, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  std::vector<double> out(3 * (size_t)KK);
  if ((rc = hip_ok(hipMemcpy(out.data(), s->dbuf + 1, out.size() * sizeof(double), hipMemcpyDeviceToHost), "D2H")))
    return rc;
  cpR.assign(out.begin(), out.begin() + KK);
  hRT.assign(out.begin() + KK, out.begin() + 2 * KK);
  sR.assign(out.begin() + 2 * KK, out.end());
  return CKMI_OK;
}

// wdot[KK], mixture cp and h (per mass) at one (T, P, Y) state (ckmi_rop_thermo, n = 1)
int rop_state(ChemSet* s, double T, double P, const double* Y, double* wdot, double* cp, double* h) {
  const int KK = s->KK;
  int rc = ensure_scratch(s, 2 + 2 * (size_t)KK + 2);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  std::vector<double> in(2 + KK);
  in[0] = T;
  in[1] = P;
  std::copy(Y, Y + KK, in.begin() + 2);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  double* o = s->dbuf + 2 + KK;
  rc = ckmi_rop_thermo(s->mech, 1, s->dbuf, s->dbuf + 1, s->dbuf + 2, o, o + KK, o + KK + 1, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  std::vector<double> out(KK + 2);
  if ((rc = hip_ok(hipMemcpy(out.data(), o, out.size() * sizeof(double), hipMemcpyDeviceToHost), "D2H"))) return rc;
  if (wdot) std::copy(out.begin(), out.begin() + KK, wdot);
  if (cp) *cp = out[KK];
  if (h) *h = out[KK + 1];
  return CKMI_OK;
}

std::vector<double> save_times(double t_end, double dtsv) {
  // 0, dt, 2 dt, ... accumulated like the Python run() (batchreactor.py save_times), ending at t_end
  std::vector<double> t{0.0};
  double tc = 0.0;
  while (tc + dtsv < t_end * (1.0 - 1e-12)) {
    tc += dtsv;
    t.push_back(tc);
  }
  t.push_back(t_end);
  return t;
}

double value_of(const std::string& v, bool* ok) {
  char* end = nullptr;
  const double x = std::strtod(v.c_str(), &end);
  *ok = end && end != v.c_str() && trim(std::string(end)).empty();
  return x;
}

int species_index(const ChemSet* s, const std::string& name) {
  const std::string u = upper(trim(name));
  for (int k = 0; k < (int)s->names.size(); ++k)
    if (upper(s->names[k]) == u) return k;
  return -1;
}

// The one keyword policy of both front-ends (this KIN ABI and the Python drop-in's reactor_cfg,
// which asks ckmi_kin_keyword_class): keywords that set a ckmi_reactor_cfg field, keywords accepted
// without effect on the device path (print interval, volume / area given elsewhere, output files),
// and everything else rejected with a message.
const char* const KW_DEVICE[] = {"ATOL", "RTOL", "HO", "STPT", "NNEG", "TIFP", "DTIGN", "TLIM", "KLIM", "IGN_STOP",
                                 "DTSV", "ADAP", "ASTEPS", "AVAR", "AVALUE", "GFAC", "QLOS", "HTC", "TAMB", "AREAQ",
                                 "MAXIT", "NSTP", "DXMX", "POLEN", "ICHX", "GVEL", "CYBAR", "PSBAR", "DEGSAVE"};
// RTIME (residence time output), MOMEN (the momentum equation is always on unless PPRO is given) and
// AREAF (the flow area comes with KINAll0D_SetupPFRInputs' diameter) are the plug-flow reactor's
// DEGPRINT (engine text-output interval) is the engine's
const char* const KW_NOEFFECT[] = {"DELT", "VOL", "AREA", "NADAP", "NO_SDOUTPUT_WRITE", "NO_XMLOUTPUT_WRITE",
                                   "RTIME", "MOMEN", "AREAF", "DEGPRINT"};
int keyword_class(const std::string& k) {
  for (const char* x : KW_DEVICE)
    if (k == x) return 1;
  for (const char* x : KW_NOEFFECT)
    if (k == x) return 2;
  return 0;
}

// Keyword text (reactormodel.py:349-372: "KEY    value", or "KEY" for booleans) -> ckmi_reactor_cfg.
// Unknown keywords are errors (the reference's library rejects what it does not know).
int apply_keywords(const ChemSet* s, ckmi_reactor_cfg& c, double& dtsv, bool& adap) {
  for (const auto& kv : g_r.kw) {
    if (!keyword_class(kv.first))
      return fail(CKMI_ERR_UNSUPPORTED, "keyword " + kv.first + " is not supported on the device path");
    const std::string& k = kv.first;
    const std::string& v = kv.second;
    bool ok = true;
    auto num = [&](double& dst) {
      dst = value_of(v, &ok);
      return ok;
    };
    double x = 0.0;
    if (k == "ATOL") ok = num(c.atol);
    else if (k == "RTOL") ok = num(c.rtol);
    else if (k == "HO") ok = num(c.h0);
    else if (k == "STPT" || k == "DXMX") ok = num(c.hmax);
    else if (k == "NNEG") c.nneg = 1;
    else if (k == "TIFP") c.ign_mode = 1;
    else if (k == "DTIGN") { c.ign_mode = 2; ok = num(c.ign_val); }
    else if (k == "TLIM") { c.ign_mode = 3; ok = num(c.ign_val); }
    else if (k == "KLIM") {
      c.ign_mode = 4;
      c.ign_species = species_index(s, v);
      ok = c.ign_species >= 0;
    } else if (k == "IGN_STOP") c.ign_stop = 1;
    else if (k == "DTSV") ok = num(dtsv) && dtsv > 0.0;
    else if (k == "DELT" || k == "VOL" || k == "AREA" || k == "NADAP" || k == "NO_SDOUTPUT_WRITE" ||
             k == "NO_XMLOUTPUT_WRITE")
      ok = v.empty() || num(x);  // print interval, volume / area (given by SetupBatchInputs), output files
    else if (k == "RTIME" || k == "MOMEN") {  // plug flow: residence time output; momentum equation
      const std::string u = upper(trim(v));
      ok = g_r.problem == 3 && (u.empty() || u == "ON" || (k == "MOMEN" && u == "OFF"));
    } else if (k == "AREAF") ok = g_r.problem == 3 && num(x) && x > 0.0;  // the area comes with the diameter
    else if (k == "ADAP") adap = true;
    else if (k == "ASTEPS") { ok = num(x) && x >= 1.0; c.asteps = (int)x; }
    else if (k == "AVAR") {
      const std::string u = upper(trim(v));
      c.avar = (u == "T" || u == "TEMP" || u == "TEMPERATURE") ? 0 : 1 + species_index(s, v);
      ok = c.avar >= 0;
    } else if (k == "AVALUE") ok = num(c.avalue);
    else if (k == "GFAC") ok = num(c.gfac);
    else if (k == "QLOS") ok = num(c.qloss);
    else if (k == "HTC") ok = num(c.htc);
    else if (k == "TAMB") ok = num(c.tamb);
    else if (k == "AREAQ") ok = num(c.areaq);
    else if (k == "MAXIT" || k == "NSTP") { ok = num(x) && x >= 1.0; c.max_steps = (int)x; }
    else if (k == "DEGPRINT") ok = g_r.problem == 4 && num(x) && x > 0.0;
    else if (k == "DEGSAVE") ok = g_r.problem == 4 && num(x) && x > 0.0 && ((dtsv = x / (6.0 * g_r.eng[CKMI_ENG_RPM])), true);
    else if (k == "POLEN") ok = g_r.problem == 4 && num(c.eng[CKMI_ENG_POLEN]);
    else if (k == "CYBAR") ok = g_r.problem == 4 && num(c.eng[CKMI_ENG_CYBAR]) && c.eng[CKMI_ENG_CYBAR] > 0.0;
    else if (k == "PSBAR") ok = g_r.problem == 4 && num(c.eng[CKMI_ENG_PSBAR]) && c.eng[CKMI_ENG_PSBAR] > 0.0;
    else if (k == "ICHX" || k == "GVEL") {  // "ICHX a b c Twall" (engine.py:898-924), "GVEL C11 C12 C2 swirl"
      std::istringstream is(v);
      double q[4];
      int m = 0;
      while (m < 4 && (is >> q[m])) ++m;
      std::string extra;
      ok = g_r.problem == 4 && m == 4 && !(is >> extra);
      if (ok && k == "ICHX") {
        c.eng[CKMI_ENG_HTMODEL] = 1.0;
        std::copy(q, q + 3, c.eng + CKMI_ENG_HTA);
        c.eng[CKMI_ENG_TWALL] = q[3];
      } else if (ok) {
        std::copy(q, q + 4, c.eng + CKMI_ENG_C11);
      }
    } else return fail(CKMI_ERR_UNSUPPORTED, "keyword " + k + " is not supported on the device path");
    if (!ok) return fail(CKMI_ERR_ARG, "bad value for keyword " + k + ": '" + v + "'");
  }
  if (adap && c.asteps == 0 && c.avar < 0) c.asteps = 20;  // ADAP default ASTEPS (batchreactor.py:373-460)
  if (!adap) c.asteps = 0, c.avar = -1;
  return CKMI_OK;
}

int apply_profiles(ckmi_reactor_cfg& c) {
  for (const Profile& p : g_r.prof) {
    const int np = (int)p.x.size();
    if (np < 1 || np > 64) return fail(CKMI_ERR_ARG, "profile " + p.key + " must have 1..64 points");
    if (p.key == "VPRO" || p.key == "PPRO" || p.key == "TPRO") {
      if (p.key == "VPRO" && g_r.problem != 2) return fail(CKMI_ERR_ARG, "VPRO needs a given-volume (CONV) reactor");
      if (p.key == "PPRO" && g_r.problem != 1 && g_r.problem != 3)
        return fail(CKMI_ERR_ARG, "PPRO needs a given-pressure (CONP) or plug-flow reactor");
      if (p.key == "TPRO" && g_r.energy != 2) return fail(CKMI_ERR_ARG, "TPRO needs a fixed-temperature reactor");
      c.nprof = np;
      c.prof_kind = p.key == "TPRO" ? 1 : 0;
      // plug flow integrates in x - x0 (KINAll0D_SetupPFRInputs); profile abscissae are absolute positions
      const double shift = g_r.problem == 3 ? g_r.x0 : 0.0;
      for (int i = 0; i < np; ++i) c.prof_t[i] = p.x[i] - shift;
      std::copy(p.y.begin(), p.y.end(), c.prof_v);
    } else if (p.key == "QPRO" || p.key == "AEXT") {
      // QPRO takes the second slot; AEXT the second alone, or the third beside a QPRO
      const bool q = p.key == "QPRO";
      if (q && c.nprof2 > 0 && c.prof2_kind == 2) {  // AEXT came first: move it to the third slot
        c.nprof3 = c.nprof2;
        std::copy(c.prof2_t, c.prof2_t + c.nprof2, c.prof3_t);
        std::copy(c.prof2_v, c.prof2_v + c.nprof2, c.prof3_v);
        c.nprof2 = 0;
      }
      if (!q && c.nprof2 > 0 && c.prof2_kind == 1) {
        c.nprof3 = np;
        std::copy(p.x.begin(), p.x.end(), c.prof3_t);
        std::copy(p.y.begin(), p.y.end(), c.prof3_v);
        continue;
      }
      c.nprof2 = np;
      c.prof2_kind = q ? 1 : 2;
      std::copy(p.x.begin(), p.x.end(), c.prof2_t);
      std::copy(p.y.begin(), p.y.end(), c.prof2_v);
    } else {
      return fail(CKMI_ERR_UNSUPPORTED, "profile " + p.key + " is not supported on the device path");
    }
  }
  return CKMI_OK;
}

double pwl(const std::vector<double>& x, const std::vector<double>& y, double t) {
  if (t <= x.front()) return y.front();
  if (t >= x.back()) return y.back();
  size_t j = 0;
  while (j + 2 < x.size() && t >= x[j + 1]) ++j;
  return y[j] + (y[j + 1] - y[j]) / (x[j + 1] - x[j]) * (t - x[j]);
}

// the kernel's engine_volume (ckmi_reactor.hpp) on the host, for the output volume and pressure
double engine_volume_host(const double* e, double t) {
  const double B = e[CKMI_ENG_BORE], a = 0.5 * e[CKMI_ENG_STROKE], L = e[CKMI_ENG_LOLR] * a, ee = -e[CKMI_ENG_POLEN];
  const double Ab = 0.25 * M_PI * B * B;
  const double st = std::sqrt((L + a) * (L + a) - ee * ee), sb = std::sqrt((L - a) * (L - a) - ee * ee);
  const double th = (e[CKMI_ENG_CA0] + 6.0 * e[CKMI_ENG_RPM] * t) * (M_PI / 180.0) + std::asin(ee / (L + a));
  const double u = a * std::sin(th) - ee;
  return Ab * (st - sb) / (e[CKMI_ENG_CMPR] - 1.0) + Ab * (st - (a * std::cos(th) + std::sqrt(L * L - u * u)));
}

int run_reactor(ChemSet* s) {
  const int KK = s->KK, n = KK + 1;
  ckmi_reactor_cfg c;
  std::memset(&c, 0, sizeof(c));
  c.energy = g_r.energy;
  c.t_end = g_r.t_end;
  c.atol = 1.0e-12;  // the reference's defaults (batchreactor.py:91-92)
  c.rtol = 1.0e-6;
  c.tamb = 300.0;
  c.gfac = 1.0;
  c.avar = -1;
  c.qloss = g_r.qloss;
  const bool engine = g_r.problem == 4;
  if (engine) {
    std::copy(g_r.eng, g_r.eng + 20, c.eng);
    c.eng[CKMI_ENG_C11] = 2.28, c.eng[CKMI_ENG_C12] = 0.308, c.eng[CKMI_ENG_C2] = 3.24;  // Woschni without GVEL
  }
  double dtsv = g_r.t_end / 100.0;  // default DTSV (batchreactor.py:296); engines: DEGSAVE / (6 RPM)
  bool adap = false;
  int rc = apply_keywords(s, c, dtsv, adap);
  if (!rc) rc = apply_profiles(c);
  if (rc) return rc;
  if (g_r.problem == 3) {  // MOMEN OFF means a given pressure: the PPRO profile supplies it
    for (const auto& kv : g_r.kw)
      if (kv.first == "MOMEN" && upper(trim(kv.second)) == "OFF" && !(c.nprof > 0 && c.prof_kind == 0))
        return fail(CKMI_ERR_ARG, "MOMEN OFF needs a PPRO pressure profile (the momentum equation gives the pressure otherwise)");
  }
  if (engine) {
    if (c.qloss != 0.0 || c.htc != 0.0 || c.nprof > 0 || c.nprof2 > 0)
      return fail(CKMI_ERR_UNSUPPORTED, "QLOS / HTC / profiles do not apply to an engine cylinder (use ICHX)");
    if (c.eng[CKMI_ENG_HTMODEL] == 1.0) {
      if (!s->dtran) return fail(CKMI_ERR_ARG, "ICHX needs transport data (KINPreProcess with itran = 1)");
      // CYBAR / PSBAR default to 1.0 (ChemkinKeywordTips.yaml:429-436)
      if (!(c.eng[CKMI_ENG_CYBAR] > 0.0)) c.eng[CKMI_ENG_CYBAR] = 1.0;
      if (!(c.eng[CKMI_ENG_PSBAR] > 0.0)) c.eng[CKMI_ENG_PSBAR] = 1.0;
      c.tran = s->dtran;
    }
  }
  const bool pfr = g_r.problem == 3;
  std::vector<double> ts;
  if (pfr) {
    // plug flow: DTSV [s] becomes the distance DTSV u0 between saved points, and the points are
    // 0, dx, 2 dx, ... <= the length (the reference's plugflow golden: 373 points, no end point)
    if (c.qloss != 0.0 || c.htc != 0.0 || c.nprof2 > 0)
      return fail(CKMI_ERR_UNSUPPORTED, "wall heat loss of a plug-flow reactor is not on this path");
    bool have_dtsv = false;
    for (const auto& kv : g_r.kw) have_dtsv = have_dtsv || kv.first == "DTSV";
    const double dx = have_dtsv ? dtsv * g_r.V0 : g_r.t_end / 100.0;
    for (int i = 0; i * dx <= g_r.t_end * (1.0 + 1e-12); ++i) ts.push_back(std::min(i * dx, g_r.t_end));
  } else {
    ts = save_times(g_r.t_end, dtsv);
  }
  const int nsave = (int)ts.size();
  const int max_adap = adap ? MAX_ADAP : 0;
  (void)hipSetDevice(s->device);
  // device buffers: inputs, outputs, save grid, adaptive points
  const size_t nd = 4 + KK + 4 + KK + 1 + nsave + (size_t)nsave * n + (adap ? (size_t)max_adap * (n + 1) : 0);
  double* d = nullptr;
  int32_t* di = nullptr;
  if ((rc = hip_ok(hipMalloc((void**)&d, nd * sizeof(double)), "hipMalloc"))) return rc;
  if ((rc = hip_ok(hipMalloc((void**)&di, (2 + CKMI_NSTAT) * sizeof(int32_t)), "hipMalloc"))) {
    (void)hipFree(d);
    return rc;
  }
  double *T0 = d, *P0 = d + 1, *V0 = d + 2, *Y0 = d + 4, *tau = Y0 + KK, *Te = tau + 1, *Pe = tau + 2, *Ve = tau + 3;
  double *Ye = tau + 4, *tstop = Ye + KK, *tsv = tstop + 1, *ysv = tsv + nsave, *tad = ysv + (size_t)nsave * n;
  double* yad = tad + max_adap;
  int32_t *prob = di, *nad = di + 1, *stats = di + 2;
  std::vector<double> hin(4 + KK, 0.0);
  hin[0] = g_r.T0;
  hin[1] = g_r.P0;
  hin[2] = g_r.V0 > 0.0 ? g_r.V0 : 1.0;
  std::copy(g_r.Y0.begin(), g_r.Y0.end(), hin.begin() + 4);
  const int32_t pr = g_r.problem;
  rc = hip_ok(hipMemcpy(d, hin.data(), hin.size() * sizeof(double), hipMemcpyHostToDevice), "H2D");
  if (!rc) rc = hip_ok(hipMemcpy(tsv, ts.data(), ts.size() * sizeof(double), hipMemcpyHostToDevice), "H2D");
  if (!rc) rc = hip_ok(hipMemcpy(prob, &pr, sizeof(int32_t), hipMemcpyHostToDevice), "H2D");
  ckmi_reactor_ext ext;
  std::memset(&ext, 0, sizeof(ext));
  ext.t_stop = tstop;
  if (adap) {
    ext.max_adap = max_adap;
    ext.t_adap = tad;
    ext.y_adap = yad;
    ext.n_adap = nad;
  }
  if (!rc) {
    rc = ckmi_reactor_run_ex(s->mech, &c, 1, prob, T0, P0, V0, Y0, &ext, tau, Te, Pe, Ve, Ye, stats, nsave, tsv, ysv,
                             nullptr);
    if (rc) rc = fail(rc, ckmi_last_error());
  }
  if (!rc) rc = hip_ok(hipDeviceSynchronize(), "reactor run");
  std::vector<double> out;
  std::vector<int32_t> iout(2 + CKMI_NSTAT);
  if (!rc) {
    out.resize(nd - (4 + KK));
    rc = hip_ok(hipMemcpy(out.data(), tau, out.size() * sizeof(double), hipMemcpyDeviceToHost), "D2H");
  }
  if (!rc) rc = hip_ok(hipMemcpy(iout.data(), di, iout.size() * sizeof(int32_t), hipMemcpyDeviceToHost), "D2H");
  (void)hipFree(d);
  (void)hipFree(di);
  if (rc) return rc;
  const double* o = out.data();  // relative to tau
  const int status = iout[2 + CKMI_STAT_STATUS];
  g_r.tau = o[0];
  const double t_stop = o[4 + KK];
  // solution points: the DTSV grid up to the stop time (+ the final state of an early stop),
  // merged with the adaptive points
  std::vector<std::pair<double, std::vector<double>>> pts;
  const double* ys = o + 4 + KK + 1 + nsave;
  for (int i = 0; i < nsave; ++i) {
    if (std::isnan(ys[(size_t)i * n])) continue;
    pts.push_back({ts[i], std::vector<double>(ys + (size_t)i * n, ys + (size_t)(i + 1) * n)});
  }
  if (t_stop < ts.back() && (pts.empty() || t_stop > pts.back().first)) {
    std::vector<double> yf(n);
    yf[0] = o[1];
    std::copy(o + 4, o + 4 + KK, yf.begin() + 1);
    pts.push_back({t_stop, yf});
  }
  if (adap) {
    const int na = iout[1];
    const double* ta = ys + (size_t)nsave * n;
    const double* ya = ta + max_adap;
    for (int i = 0; i < na; ++i) {
      if (ta[i] > t_stop) continue;
      bool dup = false;
      for (double x : ts) dup = dup || x == ta[i];
      if (!dup) pts.push_back({ta[i], std::vector<double>(ya + (size_t)i * n, ya + (size_t)(i + 1) * n)});
    }
    std::stable_sort(pts.begin(), pts.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  }
  // pressure and volume of every point (CONP: P given, V from the mass; CONV: V given, P from the EOS)
  double sw0 = 0.0;
  for (int k = 0; k < KK; ++k) sw0 += g_r.Y0[k] / s->wt[k];
  const Profile* pp = nullptr;
  for (const Profile& p : g_r.prof)
    if (((g_r.problem == 1 || pfr) && p.key == "PPRO") || (g_r.problem == 2 && p.key == "VPRO")) pp = &p;
  const double Vs = (g_r.problem == 2 && pp) ? pp->y.front() : hin[2];
  const double rho0 = g_r.P0 / (RU * g_r.T0 * sw0);
  g_r.t.clear(), g_r.T.clear(), g_r.P.clear(), g_r.V.clear(), g_r.Y.clear();
  for (const auto& pt : pts) {
    const double t = pt.first, T = pt.second[0];
    double sw = 0.0;
    for (int k = 0; k < KK; ++k) sw += pt.second[1 + k] / s->wt[k];
    double P, V;
    if (engine) {
      V = engine_volume_host(c.eng, t);  // c.eng: with the POLEN keyword
      P = (rho0 * engine_volume_host(c.eng, 0.0) / V) * RU * T * sw;
    } else if (pfr) {  // momentum (ckmi.h problem 3) or PPRO; V = the velocity
      // as the kernels (ckmi.hip reactor_kernel, PFR.py:609-612): the mass flux from the inlet state, the
      // PPRO profile in absolute positions (t is relative to the start position x0)
      const double G = g_r.P0 / (RU * g_r.T0 * sw0) * g_r.V0, Pm = g_r.P0 + G * g_r.V0;
      P = pp ? pwl(pp->x, pp->y, t + g_r.x0)
             : 0.5 * (Pm + std::sqrt(std::max(Pm * Pm - 4.0 * G * G * RU * T * sw, 0.0)));  // choked: status 5
      V = G / (P / (RU * T * sw));
    } else if (g_r.problem == 1) {
      P = pp ? pwl(pp->x, pp->y, t) : g_r.P0;
      V = rho0 * Vs / (P / (RU * T * sw));
    } else {
      V = pp ? pwl(pp->x, pp->y, t) : Vs;
      P = (rho0 * Vs / V) * RU * T * sw;
    }
    g_r.t.push_back(pfr ? g_r.x0 + t : t);
    g_r.T.push_back(T);
    g_r.P.push_back(P);
    g_r.V.push_back(V);
    g_r.Y.insert(g_r.Y.end(), pt.second.begin() + 1, pt.second.end());
  }
  g_r.cfg = c;
  g_r.done = true;
  if (status != CKMI_RUN_OK)
    return fail(100 + status, "reactor integration failed (status " + std::to_string(status) + ")");
  return CKMI_OK;
}

int register_set(const ckmi_mech_desc* desc, int32_t MM, const char* names, const char* elements,
                 const double* awt, const int32_t* ncf, int32_t* chemset, ChemSet** out) {
  if (!desc || !chemset || MM < 0) return fail(CKMI_ERR_ARG, "null argument");
  auto* s = new ChemSet();
  ckmi_mech_desc dd = *desc;  // the element counts also drive the reactors' element projection
  if (!dd.ncf && ncf && MM > 0) {
    dd.MM = MM;
    dd.ncf = ncf;
  }
  int rc = ckmi_mech_create(&dd, &s->mech);
  if (rc) {
    delete s;
    return fail(rc, ckmi_last_error());
  }
  (void)hipGetDevice(&s->device);
  s->KK = desc->KK;
  s->II = desc->II;
  s->wt.assign(desc->wt, desc->wt + desc->KK);
  s->thermo.assign(desc->thermo, desc->thermo + 17 * (size_t)desc->KK);
  s->MM = (awt && ncf) ? MM : 0;
  if (s->MM) {
    s->awt.assign(awt, awt + MM);
    s->ncf.assign(ncf, ncf + (size_t)MM * desc->KK);
  }
  for (int k = 0; names && k < s->KK; ++k)
    s->names.emplace_back(trim(std::string(names + NAME_LEN * k, strnlen(names + NAME_LEN * k, NAME_LEN))));
  for (int m = 0; elements && m < MM; ++m)
    s->elements.emplace_back(trim(std::string(elements + NAME_LEN * m, strnlen(elements + NAME_LEN * m, NAME_LEN))));
  g_sets.push_back(s);
  *chemset = (int32_t)g_sets.size();
  g_active = *chemset;
  if (out) *out = s;
  return CKMI_OK;
}

}  // namespace

extern "C" {

const char* ckmi_kin_last_error(void) { return g_err.c_str(); }

int ckmi_kin_keyword_class(const char* key) { return key ? keyword_class(upper(trim(key))) : 0; }

int ckmi_kin_register(const ckmi_mech_desc* desc, int32_t MM, const char* names, const char* elements,
                      const double* awt, const int32_t* ncf, int32_t* chemset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return register_set(desc, MM, names, elements, awt, ncf, chemset, nullptr);
}

int ckmi_kin_release(int32_t chemset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(&chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  if (s->dbuf) (void)hipFree(s->dbuf);
  ckmi_transport_destroy(s->tran);
  if (s->dtran) (void)hipFree(s->dtran);
  ckmi_mech_destroy(s->mech);
  delete s;
  g_sets[chemset - 1] = nullptr;
  return CKMI_OK;
}

int KINSetUnitSystem(int* code) {
  if (!code || *code != 1) return fail(CKMI_ERR_UNSUPPORTED, "only the cgs unit system (1) is supported");
  return CKMI_OK;
}

int KINInitialize(int* chemset, int* flag) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)flag;
  if (!get_set(chemset)) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  g_active = *chemset;
  return CKMI_OK;
}

void KINFinish(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_r = Reactor0D();
}

int KINUpdateChemistrySet(int* chemset) { return KINInitialize(chemset, nullptr); }
int KINSwitchChemistrySet(int* chemset) { return KINInitialize(chemset, nullptr); }

int KINGetChemistrySizes(int* chemset, int* MM, int* KK, int* II, int* nmat, int* nsite, int* nbulk, int* nphase,
                         int* nsurfrxn) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  if (MM) *MM = s->MM;
  if (KK) *KK = s->KK;
  if (II) *II = s->II;
  if (nmat) *nmat = 1;  // gas phase only (no surface chemistry on this path)
  if (nsite) *nsite = 0;
  if (nbulk) *nbulk = 0;
  if (nphase) *nphase = 1;
  if (nsurfrxn) *nsurfrxn = 0;
  return CKMI_OK;
}

static int copy_names(const std::vector<std::string>& v, char** out) {
  if (!out) return fail(CKMI_ERR_ARG, "null name buffers");
  for (size_t i = 0; i < v.size(); ++i) {
    if (!out[i]) return fail(CKMI_ERR_ARG, "null name buffer");
    std::memset(out[i], 0, NAME_LEN + 1);
    std::memcpy(out[i], v[i].c_str(), std::min<size_t>(v[i].size(), NAME_LEN));
  }
  return CKMI_OK;
}

int KINGetGasSpeciesNames(int* chemset, char** names) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  if ((int)s->names.size() != s->KK) return fail(CKMI_ERR_ARG, "species names were not registered");
  return copy_names(s->names, names);
}

int KINGetElementNames(int* chemset, char** names) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  if ((int)s->elements.size() != s->MM) return fail(CKMI_ERR_ARG, "element names were not registered");
  return copy_names(s->elements, names);
}

int KINGetAtomicWeights(int* chemset, double* awt) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !awt) return fail(CKMI_ERR_ARG, "bad argument");
  std::copy(s->awt.begin(), s->awt.end(), awt);
  return CKMI_OK;
}

int KINGetGasMolecularWeights(int* chemset, double* wt) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !wt) return fail(CKMI_ERR_ARG, "bad argument");
  std::copy(s->wt.begin(), s->wt.end(), wt);
  return CKMI_OK;
}

int KINGetGasSpeciesComposition(int* chemset, int32_t* ncf) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !ncf) return fail(CKMI_ERR_ARG, "bad argument");
  for (int m = 0; m < s->MM; ++m)
    for (int k = 0; k < s->KK; ++k) ncf[m + (size_t)s->MM * k] = s->ncf[(size_t)m * s->KK + k];  // F-order [MM, KK]
  return CKMI_OK;
}

// per-mass species properties from the device NASA-7 kernel
static int species_per_mass(int* chemset, double* T, double* out, int which) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !out || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  std::vector<double> cpR, hRT, sR;
  int rc = species_thermo(s, *T, cpR, hRT, sR);
  if (rc) return rc;
  for (int k = 0; k < s->KK; ++k) {
    const double r = RU / s->wt[k];
    out[k] = which == 0 ? cpR[k] * r : (which == 1 ? hRT[k] * r * *T : (hRT[k] - 1.0) * r * *T);
  }
  return CKMI_OK;
}

int KINGetGasSpecificHeat(int* chemset, double* T, double* cp) { return species_per_mass(chemset, T, cp, 0); }
int KINGetGasSpeciesEnthalpy(int* chemset, double* T, double* h) { return species_per_mass(chemset, T, h, 1); }
int KINGetGasSpeciesInternalEnergy(int* chemset, double* T, double* u) { return species_per_mass(chemset, T, u, 2); }

int KINGetMassDensity(int* chemset, double* T, double* P, double* Y, double* rho) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !P || !Y || !rho || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  double sw = 0.0;
  for (int k = 0; k < s->KK; ++k) sw += Y[k] / s->wt[k];
  *rho = *P / (RU * *T * sw);  // ideal-gas EOS (the only EOS of this path)
  return CKMI_OK;
}

int KINGetGasMixtureSpecificHeat(int* chemset, double* T, double* Y, double* cp) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !Y || !cp || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  return rop_state(s, *T, 1.01325e6, Y, nullptr, cp, nullptr);
}

int KINGetGasMixtureEnthalpy(int* chemset, double* T, double* Y, double* h) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !Y || !h || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  return rop_state(s, *T, 1.01325e6, Y, nullptr, nullptr, h);
}

int KINGetGasROP(int* chemset, double* T, double* P, double* Y, double* wdot) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !P || !Y || !wdot || !(*T > 0.0) || !(*P > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  return rop_state(s, *T, *P, Y, wdot, nullptr, nullptr);
}

int KINGetGasReactionRates(int* chemset, double* T, double* P, double* Y, double* qf, double* qr) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !P || !Y || !qf || !qr || !(*T > 0.0) || !(*P > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  const int KK = s->KK, II = s->II;
  int rc = ensure_scratch(s, 2 + (size_t)KK + 2 * (size_t)II);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  // The composition argument of this entry point is read as MOLE fractions, like Chemkin's CKKFKR
  // (P, T, X): the reference's golden (reactionrates.baseline) is reproduced to 1e-14 that way and
  // misses by up to 1.8x when the array is read as mass fractions -- although mixture.py:1540
  // passes mass fractions.  Drop-in means the same numbers, so the convention is kept here; the
  // batched ckmi_reaction_rates takes mass fractions.
  std::vector<double> in(2 + KK);
  in[0] = *T;
  in[1] = *P;
  double sxw = 0.0;
  for (int k = 0; k < KK; ++k) sxw += Y[k] * s->wt[k];
  if (!(sxw > 0.0)) return fail(CKMI_ERR_ARG, "composition sums to zero");
  for (int k = 0; k < KK; ++k) in[2 + k] = Y[k] * s->wt[k] / sxw;
  if ((rc = hip_ok(hipMemcpy(s->dbuf, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  double* o = s->dbuf + 2 + KK;
  rc = ckmi_reaction_rates(s->mech, 1, s->dbuf, s->dbuf + 1, s->dbuf + 2, o, o + II, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  if ((rc = hip_ok(hipMemcpy(qf, o, II * sizeof(double), hipMemcpyDeviceToHost), "D2H"))) return rc;
  return hip_ok(hipMemcpy(qr, o + II, II * sizeof(double), hipMemcpyDeviceToHost), "D2H");
}

int KINGetReactionRateParameters(int* chemset, double* A, double* b, double* E_R) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  const int rc = ckmi_get_arrhenius(s->mech, A, b, E_R);
  return rc ? fail(rc, ckmi_last_error()) : CKMI_OK;
}

int KINSetAFactorForAReaction(int* chemset, int* irxn, double* A) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !irxn || !A || *irxn == 0 || std::abs(*irxn) > s->II) return fail(CKMI_ERR_ARG, "bad reaction index");
  if (*irxn > 0) {  // get (1-based)
    std::vector<double> a(s->II);
    const int rc = ckmi_get_arrhenius(s->mech, a.data(), nullptr, nullptr);
    if (rc) return fail(rc, ckmi_last_error());
    *A = a[*irxn - 1];
    return CKMI_OK;
  }
  (void)hipSetDevice(s->device);
  const int rc = ckmi_set_afactor(s->mech, -*irxn - 1, *A);  // negative index: put (chemistry.py:1660-1667)
  return rc ? fail(rc, ckmi_last_error()) : CKMI_OK;
}

int KINAll0D_Setup(int* chemset, int* reactortype, int* problem, int* energy, int* solver, int* npsr,
                   int32_t* ninlets, int* nzones) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)npsr, (void)ninlets, (void)nzones;
  if (!get_set(chemset)) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  if (!reactortype || (*reactortype != 1 && *reactortype != 3 && *reactortype != 4))
    return fail(CKMI_ERR_UNSUPPORTED, "only closed batch reactors (type 1), plug-flow reactors (type 3) and "
                                      "single-zone HCCI engines (type 4)");
  if (!solver || *solver != 1) return fail(CKMI_ERR_UNSUPPORTED, "only the transient solver (1)");
  if (*reactortype == 4) {  // HCCI.py:84-139: problem ICEN (3), one zone
    if (!problem || *problem != 3) return fail(CKMI_ERR_ARG, "an HCCI engine needs problem 3 (ICEN)");
    if (nzones && *nzones != 1) return fail(CKMI_ERR_UNSUPPORTED, "multi-zone HCCI engines are not on this path");
  } else if (!problem || (*problem != 1 && *problem != 2)) {
    return fail(CKMI_ERR_ARG, "problem must be 1 (CONP) or 2 (CONV)");
  }
  if (!energy || (*energy != 1 && *energy != 2)) return fail(CKMI_ERR_ARG, "energy must be 1 (ENRG) or 2 (TGIV)");
  g_r = Reactor0D();
  g_r.chemset = *chemset;
  g_r.reactortype = *reactortype;
  // PFR.py:75 sets CONP; x is the variable (problem 3); HCCI: ckmi_reactor_run's engine problem 4
  g_r.problem = *reactortype == 3 ? 3 : (*reactortype == 4 ? 4 : *problem);
  g_r.energy = *energy;
  g_r.setup = true;
  return CKMI_OK;
}

int KINAll0D_SetupWorkArrays(int* lout, int* chemset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)lout;
  if (!get_set(chemset)) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  return CKMI_OK;  // device work arrays are allocated per run
}

int KINAll0D_SetupBatchInputs(int* chemset, double* t_end, double* T, double* P, double* V, double* qloss,
                              double* area, double* Y, double* site, double* bulk) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)area, (void)site, (void)bulk;  // reactive surface area, site / bulk fractions: no surface chemistry
  ChemSet* s = get_set(chemset);
  if (!s || !g_r.setup || *chemset != g_r.chemset) return fail(CKMI_ERR_ARG, "KINAll0D_Setup first");
  if (g_r.reactortype != 1) return fail(CKMI_ERR_ARG, "KINAll0D_SetupBatchInputs on a plug-flow reactor");
  if (!t_end || !T || !P || !Y || !(*t_end > 0.0) || !(*T > 0.0) || !(*P > 0.0))
    return fail(CKMI_ERR_ARG, "TIME, temperature and pressure must be > 0");
  g_r.t_end = *t_end;
  g_r.T0 = *T;
  g_r.P0 = *P;
  g_r.V0 = V ? *V : 0.0;
  g_r.qloss = qloss ? *qloss : 0.0;
  g_r.Y0.assign(Y, Y + s->KK);
  g_r.kw.clear();
  g_r.prof.clear();
  g_r.inputs = true;
  g_r.done = false;
  return CKMI_OK;
}

// KINAll0D_SetupPFRInputs (chemkin_wrapper.py:643-656, flowreactors/PFR.py:498-512): start position,
// end position (XEND) [cm], inlet T [K] and P [dyn/cm2], heat loss, diameter [cm], site / bulk
// fractions (no surface chemistry), inlet mass flow rate [g/s], inlet mass fractions.  The reactor
// runs as problem 3 of ckmi_reactor_run: x - x0 is the integration variable and the inlet velocity
// mdot / (rho A), A = pi d^2 / 4, the per-reactor V0.
int KINAll0D_SetupPFRInputs(int* chemset, double* x0, double* xend, double* T, double* P, double* qloss,
                            double* diam, double* site, double* bulk, double* mdot, double* Y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)site, (void)bulk;
  ChemSet* s = get_set(chemset);
  if (!s || !g_r.setup || *chemset != g_r.chemset) return fail(CKMI_ERR_ARG, "KINAll0D_Setup first");
  if (g_r.reactortype != 3) return fail(CKMI_ERR_ARG, "KINAll0D_SetupPFRInputs needs reactor type 3 (PFR)");
  if (!x0 || !xend || !T || !P || !diam || !mdot || !Y || !(*xend > *x0) || !(*T > 0.0) || !(*P > 0.0) ||
      !(*diam > 0.0) || !(*mdot > 0.0))
    return fail(CKMI_ERR_ARG, "PFR inputs: XEND > start, T, P, diameter and mass flow rate must be > 0");
  double sw = 0.0;
  for (int k = 0; k < s->KK; ++k) sw += Y[k] / s->wt[k];
  if (!(sw > 0.0)) return fail(CKMI_ERR_ARG, "PFR inlet composition sums to zero");
  const double rho = *P / (RU * *T * sw);
  const double area = 3.14159265358979323846 * *diam * *diam / 4.0;
  g_r.x0 = *x0;
  g_r.t_end = *xend - *x0;
  g_r.T0 = *T;
  g_r.P0 = *P;
  g_r.V0 = *mdot / (rho * area);
  g_r.qloss = qloss ? *qloss : 0.0;
  g_r.Y0.assign(Y, Y + s->KK);
  g_r.kw.clear();
  g_r.prof.clear();
  g_r.inputs = true;
  g_r.done = false;
  return CKMI_OK;
}

// KINAll0D_SetupHCCIInputs (chemkin_wrapper.py:657-670, HCCI.py:1105-1125): IVC and EVO crank angles
// [deg], RPM, compression ratio, bore and stroke [cm], rod length / crank radius, T [K] and P [dyn/cm2]
// at IVC, heat loss (must be 0: ICHX replaces it), mass fractions.  The cylinder runs as problem 4 of
// ckmi_reactor_run; POLEN / ICHX / GVEL / CYBAR / PSBAR / DEGSAVE come as keywords.
int KINAll0D_SetupHCCIInputs(int* chemset, double* ivc, double* evo, double* rpm, double* cmpr, double* bore,
                             double* stroke, double* lolr, double* T, double* P, double* qloss, double* Y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !g_r.setup || *chemset != g_r.chemset) return fail(CKMI_ERR_ARG, "KINAll0D_Setup first");
  if (g_r.reactortype != 4) return fail(CKMI_ERR_ARG, "KINAll0D_SetupHCCIInputs needs reactor type 4 (HCCI)");
  if (!ivc || !evo || !rpm || !cmpr || !bore || !stroke || !lolr || !T || !P || !Y || !(*evo > *ivc) ||
      !(*rpm > 0.0) || !(*cmpr > 1.0) || !(*bore > 0.0) || !(*stroke > 0.0) || !(*lolr > 1.0) || !(*T > 0.0) ||
      !(*P > 0.0))
    return fail(CKMI_ERR_ARG, "HCCI inputs: EVO > IVC, RPM, bore, stroke, T, P > 0, CMPR > 1, rod / crank > 1");
  if (qloss && *qloss != 0.0) return fail(CKMI_ERR_UNSUPPORTED, "engine heat loss comes from ICHX, not QLOS");
  if (s->KK + 1 > 64) return fail(CKMI_ERR_UNSUPPORTED, "engine cylinders need at most 63 species");
  std::fill(g_r.eng, g_r.eng + 20, 0.0);
  g_r.eng[CKMI_ENG_CA0] = *ivc;
  g_r.eng[CKMI_ENG_RPM] = *rpm;
  g_r.eng[CKMI_ENG_CMPR] = *cmpr;
  g_r.eng[CKMI_ENG_BORE] = *bore;
  g_r.eng[CKMI_ENG_STROKE] = *stroke;
  g_r.eng[CKMI_ENG_LOLR] = *lolr;
  g_r.t_end = (*evo - *ivc) / (6.0 * *rpm);
  g_r.T0 = *T;
  g_r.P0 = *P;
  g_r.V0 = 1.0;
  g_r.qloss = 0.0;
  g_r.Y0.assign(Y, Y + s->KK);
  g_r.kw.clear();
  g_r.prof.clear();
  g_r.inputs = true;
  g_r.done = false;
  return CKMI_OK;
}

// KINAll0D_GetEngineHeatRelease (chemkin_wrapper.py:769-777, engine.py:953-988) on the last engine run.
//   hr10 / hr50 / hr90: crank angles of 10 / 50 / 90 % of the cumulative chemical heat release,
//     -sum_k h_k(298.15 K) W_k (n_k(t) - n_k(0)), on the solution points (linear interpolation);
//   ahrr: the peak apparent heat-release rate per CA [erg/degree], m c_v dT/dCA + P dV/dCA from the
//     integrator's right-hand side at the solution points (ckmi_engine_heat_rates on the device);
//   ahrrp: the peak of the same from the pressure trace with the charge's constant gamma,
//     gamma/(gamma-1) P dV/dCA + 1/(gamma-1) V dP/dCA (central differences on the solution points);
//   qloss_ca[0]: the peak wall heat-loss rate per CA [erg/degree], hA (T - T_wall) (ICHX; 0 adiabatic).
// The reference reads these as scalars; which instant its library reports is not documented in the
// reference, so the peaks over the cycle are returned (the full profiles: ckmi_engine_heat_rates).
int KINAll0D_GetEngineHeatRelease(double* qloss_ca, double* ahrr, double* ahrrp, double* hr10, double* hr50,
                                  double* hr90) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_r.done || g_r.problem != 4) return fail(CKMI_ERR_ARG, "no completed engine run");
  ChemSet* s = get_set(&g_r.chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  std::vector<double> cpR, hRT, sR;
  int rc = species_thermo(s, 298.15, cpR, hRT, sR);
  if (rc) return rc;
  const int KK = s->KK, n1 = KK + 1;
  const size_t np = g_r.t.size();
  std::vector<double> q(np, 0.0);
  for (size_t i = 0; i < np; ++i)
    for (int k = 0; k < KK; ++k)
      q[i] -= (g_r.Y[i * KK + k] - g_r.Y[k]) * hRT[k] * RU * 298.15 / s->wt[k];
  const double rate = 6.0 * g_r.eng[CKMI_ENG_RPM];  // degrees per second
  // heat rates on the device, at the solution points
  std::vector<double> ah(np, 0.0), ql(np, 0.0);
  if (np > 0) {
    (void)hipSetDevice(s->device);
    std::vector<double> hin(KK + np + np * n1);
    std::copy(g_r.Y0.begin(), g_r.Y0.end(), hin.begin());
    std::copy(g_r.t.begin(), g_r.t.end(), hin.begin() + KK);
    for (size_t i = 0; i < np; ++i) {
      hin[KK + np + i * n1] = g_r.T[i];
      std::copy(g_r.Y.begin() + i * KK, g_r.Y.begin() + (i + 1) * KK, hin.begin() + KK + np + i * n1 + 1);
    }
    double* d = nullptr;
    if ((rc = hip_ok(hipMalloc((void**)&d, (hin.size() + 2 * np) * sizeof(double)), "hipMalloc"))) return rc;
    double *dY0 = d, *dt = d + KK, *dy = dt + np, *dah = dy + np * n1, *dql = dah + np;
    rc = hip_ok(hipMemcpy(d, hin.data(), hin.size() * sizeof(double), hipMemcpyHostToDevice), "H2D");
    if (!rc) {
      rc = ckmi_engine_heat_rates(s->mech, &g_r.cfg, g_r.T0, g_r.P0, dY0, (int32_t)np, dt, dy, dah, dql, nullptr);
      if (rc) rc = fail(rc, ckmi_last_error());
    }
    if (!rc) rc = hip_ok(hipDeviceSynchronize(), "engine heat rates");
    if (!rc) rc = hip_ok(hipMemcpy(ah.data(), dah, np * sizeof(double), hipMemcpyDeviceToHost), "D2H");
    if (!rc) rc = hip_ok(hipMemcpy(ql.data(), dql, np * sizeof(double), hipMemcpyDeviceToHost), "D2H");
    (void)hipFree(d);
    if (rc) return rc;
  }
  double gamma = 1.4;
  {  // gamma of the charge at IVC
    std::vector<double> c0, h0, s0;
    if ((rc = species_thermo(s, g_r.T0, c0, h0, s0))) return rc;
    double cpm = 0.0, sw = 0.0;
    for (int k = 0; k < KK; ++k) {
      cpm += g_r.Y0[k] * c0[k] / s->wt[k];
      sw += g_r.Y0[k] / s->wt[k];
    }
    gamma = cpm / (cpm - sw);
  }
  double pk_ah = 0.0, pk_ap = 0.0, pk_ql = 0.0;
  for (size_t i = 0; i < np; ++i) {
    pk_ah = std::max(pk_ah, ah[i] / rate);
    pk_ql = std::max(pk_ql, ql[i] / rate);
    if (np > 1) {  // central differences in CA (one-sided at the ends), as numpy.gradient
      const size_t a = i == 0 ? 0 : i - 1, b = i + 1 == np ? np - 1 : i + 1;
      const double dca = (g_r.t[b] - g_r.t[a]) * rate;
      const double dP = (g_r.P[b] - g_r.P[a]) / dca, dV = (g_r.V[b] - g_r.V[a]) / dca;
      pk_ap = std::max(pk_ap, gamma / (gamma - 1.0) * g_r.P[i] * dV + g_r.V[i] * dP / (gamma - 1.0));
    }
  }
  if (qloss_ca) *qloss_ca = pk_ql;
  if (ahrr) *ahrr = pk_ah;
  if (ahrrp) *ahrrp = pk_ap;
  double* out[3] = {hr10, hr50, hr90};
  const double lev[3] = {0.1, 0.5, 0.9};
  for (int j = 0; j < 3; ++j) {
    if (!out[j]) continue;
    double ca = g_r.eng[CKMI_ENG_CA0];
    if (np > 1 && q.back() > 0.0)
      for (size_t i = 1; i < np; ++i)
        if (q[i] / q.back() >= lev[j]) {
          const double f0 = q[i - 1] / q.back(), f1 = q[i] / q.back();
          const double t = g_r.t[i - 1] + (lev[j] - f0) / (f1 - f0) * (g_r.t[i] - g_r.t[i - 1]);
          ca = g_r.eng[CKMI_ENG_CA0] + t * rate;
          break;
        }
    *out[j] = ca;
  }
  return CKMI_OK;
}

int KINAll0D_IntegrateHeatRelease(void) { return CKMI_OK; }  // QRGEQ output: not produced (no KINAll0D_GetHeatRelease)

int KINAll0D_SetProfilePoints(int* npoints) {
  if (!npoints || *npoints < 0) return fail(CKMI_ERR_ARG, "bad profile size");
  return CKMI_OK;
}

int KINAll0D_SetProfileParameter(char* key, int* npoints, double* x, double* y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_r.inputs) return fail(CKMI_ERR_ARG, "KINAll0D_SetupBatchInputs first");
  if (!key || !npoints || *npoints < 1 || *npoints > 64 || !x || !y) return fail(CKMI_ERR_ARG, "bad profile");
  Profile p;
  p.key = upper(trim(key));
  p.x.assign(x, x + *npoints);
  p.y.assign(y, y + *npoints);
  for (auto& q : g_r.prof)
    if (q.key == p.key) {
      q = p;
      return CKMI_OK;
    }
  g_r.prof.push_back(p);
  return CKMI_OK;
}

int KINAll0D_SetUserKeyword(char* line) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_r.inputs) return fail(CKMI_ERR_ARG, "KINAll0D_SetupBatchInputs first");
  if (!line) return fail(CKMI_ERR_ARG, "null keyword line");
  std::string s = trim(line);
  if (s.empty() || s[0] == '!') return CKMI_OK;  // '!' disables a keyword (reactormodel.py:341-372)
  std::istringstream is(s);
  std::string key, value, rest;
  is >> key;
  std::getline(is, rest);
  value = trim(rest);
  g_r.kw.push_back({upper(key), value});
  return CKMI_OK;
}

int KINAll0D_Calculate(int* chemset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !g_r.inputs || *chemset != g_r.chemset) return fail(CKMI_ERR_ARG, "reactor is not set up");
  g_r.done = false;
  return run_reactor(s);
}

int KINAll0D_GetIgnitionDelay(double* tau) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!tau || !g_r.done) return fail(CKMI_ERR_ARG, "no completed run");
  *tau = g_r.tau;
  return CKMI_OK;
}

int KINAll0D_GetSolnResponseSize(int* nreac, int* npts) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!nreac || !npts || !g_r.done) return fail(CKMI_ERR_ARG, "no completed run");
  *nreac = 1;
  *npts = (int)g_r.t.size();
  return CKMI_OK;
}

int KINAll0D_GetGasSolnResponse(int* nreac, int* npts, int* KK, double* t, double* T, double* P, double* V,
                                double* Y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_r.done) return fail(CKMI_ERR_ARG, "no completed run");
  const int np = (int)g_r.t.size();
  ChemSet* s = get_set(&g_r.chemset);
  if (!nreac || *nreac != 1 || !npts || *npts != np || !KK || !s || *KK != s->KK)
    return fail(CKMI_ERR_SIZE, "solution size mismatch (KINAll0D_GetSolnResponseSize)");
  for (int i = 0; i < np; ++i) {
    if (t) t[i] = g_r.t[i];
    if (T) T[i] = g_r.T[i];
    if (P) P[i] = g_r.P[i];
    if (V) V[i] = g_r.V[i];
    for (int k = 0; Y && k < s->KK; ++k) Y[k + (size_t)s->KK * i] = g_r.Y[(size_t)i * s->KK + k];  // [KK, npts] F-order
  }
  return CKMI_OK;
}


}  // extern "C"

namespace {
// ---------------------------------------------------------------- transport data (TRANLIB format)
bool read_text(const char* path, std::string& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  out.clear();
  char buf[1 << 14];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
  std::fclose(f);
  return true;
}

// the lines between a "TRANSPORT [ALL]" line and the next "END" line of a mechanism file
std::string inline_transport_block(const std::string& text) {
  std::istringstream in(text);
  std::string line, out;
  bool on = false;
  while (std::getline(in, line)) {
    std::istringstream ls(line.substr(0, line.find('!')));
    std::string w;
    ls >> w;
    w = upper(w);
    if (!on) {
      if (w.rfind("TRAN", 0) == 0) on = true;
    } else if (w == "END") {
      return out;
    } else {
      out += line + "\n";
    }
  }
  return on ? out : std::string();
}

// TRANLIB records (name, geometry, eps/k, sigma, dipole, polarizability, Zrot; '!' comments; the
// first record of a species wins) -> [KK][6] in mechanism order; every species needs one.  The
// grammar of pychemkin_amd/transport.py parse_transport_text.
bool transport_params(const std::string& text, const std::vector<std::string>& names, std::vector<double>& params,
                      std::string& why) {
  std::map<std::string, std::vector<double>> rec;
  std::istringstream in(text);
  std::string line;
  int ln = 0;
  while (std::getline(in, line)) {
    ++ln;
    std::istringstream ls(line.substr(0, line.find('!')));
    std::vector<std::string> tok;
    std::string w;
    while (ls >> w) tok.push_back(w);
    if (tok.empty()) continue;
    const std::string key = upper(tok[0]);
    if (key.rfind("TRAN", 0) == 0 || key == "END") continue;
    if (tok.size() < 7) {
      why = "transport line " + std::to_string(ln) + ": expected 7 fields";
      return false;
    }
    std::vector<double> v(6);
    for (int j = 0; j < 6; ++j) {
      char* e = nullptr;
      v[j] = std::strtod(tok[1 + j].c_str(), &e);
      if (!e || *e) {
        why = "transport line " + std::to_string(ln) + ": bad number " + tok[1 + j];
        return false;
      }
    }
    if (v[0] != 0.0 && v[0] != 1.0 && v[0] != 2.0) {
      why = "transport line " + std::to_string(ln) + ": geometry must be 0, 1 or 2";
      return false;
    }
    rec.emplace(key, v);
  }
  params.assign(6 * names.size(), 0.0);
  for (size_t k = 0; k < names.size(); ++k) {
    auto it = rec.find(upper(names[k]));
    if (it == rec.end()) {
      why = "no transport data for species " + names[k];
      return false;
    }
    std::copy(it->second.begin(), it->second.end(), params.begin() + 6 * k);
  }
  return true;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- mechanism preprocessing
// KINPreProcess (chemkin_wrapper.py:303-316, chemistry.py:675-687): parse chem.inp + therm.dat with
// the native interpreter (ckmi_parse.cpp), build the device tables and return the chemistry-set
// index.  Surface chemistry is out of scope (isurf must be 0).  With itran = 1 the transport data
// come from the transport file, or, when it does not exist, from the TRANSPORT block of the
// mechanism file (chemistry.py:450-480 preprocess_transportdata); their viscosity fits are made
// here (ckmi_transport_fit) and uploaded with the mechanism (KINGetViscosity /
// KINGetMixtureViscosity).  The summary file, when named, receives the element / species /
// reaction listing; the link files of the closed library are not written (the tables stay in this
// process).
int KINPreProcess(int* isurf, int* itran, char* chem, char* surf, char* therm, char* tran, char* gaslink,
                  char* surflink, char* tranlink, char* summary, int* chemset) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)surf, (void)gaslink, (void)surflink, (void)tranlink;
  if (!chem || !chemset) return fail(CKMI_ERR_ARG, "KINPreProcess: null mechanism file or chemistry-set pointer");
  if (isurf && *isurf != 0) return fail(CKMI_ERR_UNSUPPORTED, "surface chemistry is not supported on this path");
  std::string tran_text;
  if (itran && *itran != 0) {
    if (tran && *tran && read_text(tran, tran_text)) {
    } else {
      std::string chem_text;
      if (!read_text(chem, chem_text)) return fail(CKMI_ERR_ARG, std::string("cannot read mechanism file ") + chem);
      tran_text = inline_transport_block(chem_text);
      if (tran_text.empty())
        return fail(CKMI_ERR_ARG, std::string("KINPreProcess: transport requested, but neither the transport file ") +
                                      (tran ? tran : "") + " nor a TRANSPORT block in the mechanism file exists");
    }
  }
  ckmi_parsed* p = nullptr;
  int rc = ckmi_parse_files(chem, therm, &p);
  if (rc) return fail(rc, std::string("KINPreProcess: ") + ckmi_parse_last_error());
  int32_t MM = 0, KK = 0, II = 0;
  ckmi_parsed_sizes(p, &MM, &KK, &II);
  ckmi_mech_desc d;
  ckmi_parsed_desc(p, &d);
  std::vector<char> names((size_t)KK * NAME_LEN + 1), elems((size_t)MM * NAME_LEN + 1);
  std::vector<double> awt(MM);
  std::vector<int32_t> ncf((size_t)MM * KK);
  ckmi_parsed_symbols(p, names.data(), elems.data(), awt.data(), ncf.data());
  ChemSet* s = nullptr;
  int32_t cs = 0;
  rc = register_set(&d, MM, names.data(), elems.data(), awt.data(), ncf.data(), &cs, &s);
  if (!rc) {
    for (int i = 0; i < II; ++i) {
      int32_t len = 0;
      ckmi_parsed_equation(p, i, nullptr, 0, &len);
      std::vector<char> b((size_t)len + 1);
      ckmi_parsed_equation(p, i, b.data(), len + 1, nullptr);
      s->equations.emplace_back(b.data());
    }
  }
  ckmi_parsed_free(p);
  if (rc) return rc;
  if (!tran_text.empty()) {
    std::vector<double> params;
    std::string why;
    if (!transport_params(tran_text, s->names, params, why)) {
      ckmi_kin_release(cs);
      return fail(CKMI_ERR_ARG, "KINPreProcess: " + why);
    }
    std::vector<double> fits((size_t)4 * KK);
    rc = ckmi_transport_fit(KK, s->wt.data(), params.data(), CKMI_VISC_FIT_TLOW, CKMI_VISC_FIT_THIGH, fits.data());
    if (!rc) rc = ckmi_transport_create(s->mech, fits.data(), &s->tran);
    std::vector<double> cfits((size_t)4 * KK), f8((size_t)8 * KK);
    if (!rc) rc = ckmi_conductivity_fit(KK, s->wt.data(), params.data(), s->thermo.data(), CKMI_VISC_FIT_TLOW,
                                        CKMI_VISC_FIT_THIGH, cfits.data());
    if (!rc) rc = ckmi_transport_set_conductivity(s->tran, cfits.data());
    if (!rc) {
      for (int k = 0; k < KK; ++k) {
        std::copy(fits.begin() + 4 * k, fits.begin() + 4 * k + 4, f8.begin() + 8 * k);
        std::copy(cfits.begin() + 4 * k, cfits.begin() + 4 * k + 4, f8.begin() + 8 * k + 4);
      }
      rc = hip_ok(hipMalloc((void**)&s->dtran, f8.size() * sizeof(double)), "hipMalloc");
      if (!rc) rc = hip_ok(hipMemcpy(s->dtran, f8.data(), f8.size() * sizeof(double), hipMemcpyHostToDevice), "H2D");
    }
    if (rc) {
      const std::string msg = ckmi_last_error();
      ckmi_kin_release(cs);
      return fail(rc, "KINPreProcess: " + msg);
    }
  }
  *chemset = cs;
  if (summary && *summary) {
    FILE* f = std::fopen(summary, "w");
    if (f) {
      std::fprintf(f, "ckmi mechanism summary: %s\n  thermo: %s\n  elements %d, species %d, reactions %d\n\n", chem,
                   therm ? therm : "(inline)", MM, KK, II);
      for (int m = 0; m < MM; ++m) std::fprintf(f, "  element %3d %-16s %12.5f\n", m + 1, s->elements[m].c_str(), s->awt[m]);
      for (int k = 0; k < KK; ++k) std::fprintf(f, "  species %3d %-16s %12.5f\n", k + 1, s->names[k].c_str(), s->wt[k]);
      for (int i = 0; i < II; ++i) std::fprintf(f, "  reaction %4d %s\n", i + 1, s->equations[i].c_str());
      std::fclose(f);
    }
  }
  return CKMI_OK;
}

// KINGetViscosity (chemkin_wrapper.py:407-412, mixture.py:1860-1883): species viscosities
// [g/(cm s)] at T from the fits made by KINPreProcess (itran = 1)
int KINGetViscosity(int* chemset, double* T, double* visc) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !visc || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  if (!s->tran) return fail(CKMI_ERR_ARG, "no transport data processed (KINPreProcess with itran = 1)");
  const int KK = s->KK;
  int rc = ensure_scratch(s, 1 + (size_t)KK);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, T, sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  rc = ckmi_species_viscosity(s->tran, 1, s->dbuf, s->dbuf + 1, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  return hip_ok(hipMemcpy(visc, s->dbuf + 1, KK * sizeof(double), hipMemcpyDeviceToHost), "D2H");
}

// KINGetMixtureViscosity (chemkin_wrapper.py:442-448, mixture.py:1943-1977): Wilke mixture
// viscosity [g/(cm s)].  The composition argument is read as MASS fractions, as mixture.py:1967
// passes them (the CONV golden's state-viscocity is reproduced to <= 5e-4 that way and misses by
// 1.3 % when the array is read as mole fractions; tests/test_transport.py).
int KINGetMixtureViscosity(int* chemset, double* T, double* Y, double* visc) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !Y || !visc || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  if (!s->tran) return fail(CKMI_ERR_ARG, "no transport data processed (KINPreProcess with itran = 1)");
  const int KK = s->KK;
  int rc = ensure_scratch(s, 2 + (size_t)KK);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  std::vector<double> in(1 + KK);
  in[0] = *T;
  std::copy(Y, Y + KK, in.begin() + 1);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  rc = ckmi_mixture_viscosity(s->tran, 1, s->dbuf, s->dbuf + 1, s->dbuf + 1 + KK, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  return hip_ok(hipMemcpy(visc, s->dbuf + 1 + KK, sizeof(double), hipMemcpyDeviceToHost), "D2H");
}

// KINGetConductivity (chemkin_wrapper.py:413-418, mixture.py:1885-1909, chemistry.py:1361-1396):
// species thermal conductivities [erg/(cm s K)] at T from the fits made by KINPreProcess (itran = 1)
int KINGetConductivity(int* chemset, double* T, double* cond) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !cond || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  if (!s->tran) return fail(CKMI_ERR_ARG, "no transport data processed (KINPreProcess with itran = 1)");
  const int KK = s->KK;
  int rc = ensure_scratch(s, 1 + (size_t)KK);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, T, sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  rc = ckmi_species_conductivity(s->tran, 1, s->dbuf, s->dbuf + 1, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  return hip_ok(hipMemcpy(cond, s->dbuf + 1, KK * sizeof(double), hipMemcpyDeviceToHost), "D2H");
}

// KINGetMixtureConductivity (chemkin_wrapper.py:449-455, mixture.py:1979-2013): mixture-averaged
// conductivity [erg/(cm s K)], (sum X lambda + 1 / sum X / lambda) / 2.  The composition argument is
// read as MASS fractions, as mixture.py:2002 passes self.Y (the same convention as
// KINGetMixtureViscosity, which the CONV golden decides).
int KINGetMixtureConductivity(int* chemset, double* T, double* Y, double* cond) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !Y || !cond || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  if (!s->tran) return fail(CKMI_ERR_ARG, "no transport data processed (KINPreProcess with itran = 1)");
  const int KK = s->KK;
  int rc = ensure_scratch(s, 2 + (size_t)KK);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  std::vector<double> in(1 + KK);
  in[0] = *T;
  std::copy(Y, Y + KK, in.begin() + 1);
  if ((rc = hip_ok(hipMemcpy(s->dbuf, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice), "H2D"))) return rc;
  rc = ckmi_mixture_conductivity(s->tran, 1, s->dbuf, s->dbuf + 1, s->dbuf + 1 + KK, nullptr);
  if (rc) return fail(rc, ckmi_last_error());
  return hip_ok(hipMemcpy(cond, s->dbuf + 1 + KK, sizeof(double), hipMemcpyDeviceToHost), "D2H");
}

// KINGetGasReactionString (chemkin_wrapper.py:365-371, chemistry.py:1759-1781): 1-based reaction index
int KINGetGasReactionString(int* chemset, int* irxn, int* len, char* buf) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !irxn || !len || !buf) return fail(CKMI_ERR_ARG, "bad argument");
  if (*irxn < 1 || *irxn > s->II) return fail(CKMI_ERR_ARG, "reaction index out of range");
  if ((int)s->equations.size() != s->II)
    return fail(CKMI_ERR_UNSUPPORTED, "reaction strings are only kept for chemistry sets made by KINPreProcess");
  const std::string& e = s->equations[*irxn - 1];
  std::memcpy(buf, e.data(), e.size());  // the caller's buffer is 1024 bytes (chemistry.py:1761)
  *len = (int)e.size();
  return CKMI_OK;
}

// KINGetReactionStringLength (:372-373): the longest reaction string of the active chemistry set
int KINGetReactionStringLength(int* len) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(&g_active);
  if (!len || !s) return fail(CKMI_ERR_ARG, "no active chemistry set");
  size_t n = 0;
  for (const auto& e : s->equations) n = std::max(n, e.size());
  *len = (int)n;
  return CKMI_OK;
}

// ---------------------------------------------------------------- real-gas EOS: ideal gas only
// (chemkin_wrapper.py:545-581; chemistry.py:755-792 and realgaseos.py:30-52 read mode 0 as "ideal")
int KINRealGas_GetEOSMode(int* chemset, int* mode, char* name) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!get_set(chemset) || !mode) return fail(CKMI_ERR_ARG, "bad argument");
  *mode = 0;
  if (name) std::memcpy(name, "IDEAL", 6);  // the caller's buffer is MAX_SPECIES_LENGTH (17) bytes
  return CKMI_OK;
}
int KINRealGas_CheckRealGasStatus(int* chemset, int* mode) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!get_set(chemset) || !mode) return fail(CKMI_ERR_ARG, "bad argument");
  *mode = 0;
  return CKMI_OK;
}
int KINRealGas_UseIdealGasLaw(int* chemset, int* flag) {
  (void)flag;
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return get_set(chemset) ? CKMI_OK : fail(CKMI_ERR_ARG, "unknown chemistry set");
}
int KINRealGas_SetCurrentPressure(int* chemset, double* P) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!get_set(chemset) || !P || !(*P > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  return CKMI_OK;  // the ideal-gas EOS does not depend on it
}
int KINRealGas_UseCubicEOS(int* chemset, int* mode) {
  (void)chemset, (void)mode;
  return fail(CKMI_ERR_UNSUPPORTED, "real-gas cubic EOS is not supported on this path (ideal gas only)");
}
int KINRealGas_SetMixingRule(int* chemset, int* rule, int* flag) {
  (void)chemset, (void)rule, (void)flag;
  return fail(CKMI_ERR_UNSUPPORTED, "real-gas mixing rules are not supported on this path (ideal gas only)");
}
int KINRealGas_SetParameter(char* key, double* value) {
  (void)key, (void)value;
  return fail(CKMI_ERR_UNSUPPORTED, "real-gas parameters are not supported on this path (ideal gas only)");
}

// ---------------------------------------------------------------- small host utilities
// KINGetGamma (:582-588): cp / cv of the mixture (ideal gas: cv = cp - R / W)
int KINGetGamma(int* chemset, double* T, double* Y, double* gamma) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !T || !Y || !gamma || !(*T > 0.0)) return fail(CKMI_ERR_ARG, "bad argument");
  double cp = 0.0;
  int rc = rop_state(s, *T, 1.01325e6, Y, nullptr, &cp, nullptr);
  if (rc) return rc;
  double sw = 0.0;
  for (int k = 0; k < s->KK; ++k) sw += Y[k] / s->wt[k];
  *gamma = cp / (cp - RU * sw);
  return CKMI_OK;
}
// KINGetMassFractionFromMoleFraction / KINGetMoleFractionFromMassFraction (:855-867)
int KINGetMassFractionFromMoleFraction(int* chemset, double* X, double* Y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !X || !Y) return fail(CKMI_ERR_ARG, "bad argument");
  double sum = 0.0;
  for (int k = 0; k < s->KK; ++k) sum += X[k] * s->wt[k];
  if (!(sum > 0.0)) return fail(CKMI_ERR_ARG, "composition sums to zero");
  for (int k = 0; k < s->KK; ++k) Y[k] = X[k] * s->wt[k] / sum;
  return CKMI_OK;
}
int KINGetMoleFractionFromMassFraction(int* chemset, double* Y, double* X) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  ChemSet* s = get_set(chemset);
  if (!s || !X || !Y) return fail(CKMI_ERR_ARG, "bad argument");
  double sum = 0.0;
  for (int k = 0; k < s->KK; ++k) sum += Y[k] / s->wt[k];
  if (!(sum > 0.0)) return fail(CKMI_ERR_ARG, "composition sums to zero");
  for (int k = 0; k < s->KK; ++k) X[k] = Y[k] / s->wt[k] / sum;
  return CKMI_OK;
}

// ---------------------------------------------------------------- 0-D reactor: API-mode setters
// Declared by the reference (:702-743) but reached only as keyword text there; each maps onto the
// keyword it stands for, so both spellings end in the same ckmi_reactor_cfg field.
static int add_kw(const char* key, double v) {
  if (!g_r.inputs) return fail(CKMI_ERR_ARG, "KINAll0D_SetupBatchInputs first");
  char b[64];
  std::snprintf(b, sizeof(b), "%.17g", v);
  g_r.kw.push_back({key, b});
  return CKMI_OK;
}
int KINAll0D_SetHeatTransfer(double* htc, double* tamb) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!htc || !tamb) return fail(CKMI_ERR_ARG, "bad argument");
  int rc = add_kw("HTC", *htc);
  return rc ? rc : add_kw("TAMB", *tamb);
}
int KINAll0D_SetHeatTransferArea(double* area) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return area ? add_kw("AREAQ", *area) : fail(CKMI_ERR_ARG, "bad argument");
}
int KINAll0D_SetSolverInitialStepTime(double* h0) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return h0 ? add_kw("HO", *h0) : fail(CKMI_ERR_ARG, "bad argument");
}
int KINAll0D_SetSolverMaximumStepTime(double* hmax) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return hmax ? add_kw("STPT", *hmax) : fail(CKMI_ERR_ARG, "bad argument");
}
int KINAll0D_SetSolverMaximumIteration(int* n) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  return n ? add_kw("MAXIT", (double)*n) : fail(CKMI_ERR_ARG, "bad argument");
}
int KINAll0D_SetRelaxIteration(void) {
  return fail(CKMI_ERR_UNSUPPORTED, "relaxation iterations (steady-state solvers) are not on this path");
}
int KINAll0D_SetMinimumSpeciesBound(double* v) {
  (void)v;
  return fail(CKMI_ERR_UNSUPPORTED, "a species lower bound other than NNEG is not supported on this path");
}
int KINAll0D_SetProfileKeyword(int* a, int* b, char* key, int* n, double* x, double* y) {
  (void)a, (void)b;
  return KINAll0D_SetProfileParameter(key, n, x, y);
}

// KINAll0D_GetSolution (:739-744, PSR.py:818): the final state (T, P, mass fractions)
int KINAll0D_GetSolution(double* T, double* P, double* Y) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_r.done || g_r.t.empty()) return fail(CKMI_ERR_ARG, "no completed run");
  ChemSet* s = get_set(&g_r.chemset);
  if (!s) return fail(CKMI_ERR_ARG, "unknown chemistry set");
  const size_t last = g_r.t.size() - 1;
  if (T) *T = g_r.T[last];
  if (P) *P = g_r.P[last];
  if (Y) std::copy(g_r.Y.begin() + last * s->KK, g_r.Y.begin() + (last + 1) * s->KK, Y);
  return CKMI_OK;
}

// KINAll0D_CalculateInput (:690-697; batchreactor.py:944-978): the full-keyword mode.  The keyword
// block is one string cut by linelen[]; the lines are those of __process_keywords_withFullInputs
// (batchreactor.py:822-925): TRAN, CONP|CONV, ENRG|TGIV, PRES [atm], TEMP, TIME, REAC sp x (mole
// fractions), VOL, profile points "VPRO t v" (PPRO in atm), QRGEQ, END, and the solver / output /
// ignition keywords of API mode.  They override what KINAll0D_Setup / SetupBatchInputs gave.
int KINAll0D_CalculateInput(int* lout, int* chemset, char* lines, int* nlines, int32_t* linelen) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  (void)lout;
  ChemSet* s = get_set(chemset);
  if (!s || !lines || !nlines || *nlines < 0 || (*nlines > 0 && !linelen)) return fail(CKMI_ERR_ARG, "bad argument");
  if (!g_r.setup || g_r.chemset != *chemset) return fail(CKMI_ERR_ARG, "KINAll0D_Setup first");
  if (!g_r.inputs) {  // everything may come from the keyword block
    g_r.Y0.assign(s->KK, 0.0);
    g_r.kw.clear();
    g_r.prof.clear();
    g_r.inputs = true;
  }
  std::vector<double> X(s->KK, 0.0);
  bool have_x = false;
  size_t off = 0;
  for (int i = 0; i < *nlines; ++i) {
    if (linelen[i] < 0) return fail(CKMI_ERR_ARG, "negative keyword line length");
    const std::string line = trim(std::string(lines + off, (size_t)linelen[i]));
    off += (size_t)linelen[i];
    if (line.empty() || line[0] == '!') continue;
    std::istringstream is(line);
    std::string key;
    is >> key;
    key = upper(key);
    std::vector<std::string> v;
    for (std::string t; is >> t;) v.push_back(t);
    bool ok = true;
    auto val = [&](size_t j) {
      bool o = false;
      const double x = j < v.size() ? value_of(v[j], &o) : 0.0;
      ok = ok && o;
      return x;
    };
    if (key == "END") break;
    if (key == "TRAN" || key == "QRGEQ") continue;
    if (key == "STST") return fail(CKMI_ERR_UNSUPPORTED, "steady-state solver (STST) is not on this path");
    if (key == "CONP" || key == "CONV") g_r.problem = key == "CONP" ? 1 : 2;
    else if (key == "ENRG" || key == "TGIV") g_r.energy = key == "ENRG" ? 1 : 2;
    else if (key == "PRES") g_r.P0 = val(0) * 1.01325e6;
    else if (key == "TEMP") g_r.T0 = val(0);
    else if (key == "TIME") g_r.t_end = val(0);
    else if (key == "VOL") g_r.V0 = val(0);
    else if (key == "QLOS") g_r.qloss = val(0);
    else if (key == "REAC") {
      const int k = v.empty() ? -1 : species_index(s, v[0]);
      if (k < 0) return fail(CKMI_ERR_ARG, "REAC: unknown species in '" + line + "'");
      X[k] = val(1);
      have_x = true;
    } else if (key == "VPRO" || key == "PPRO" || key == "TPRO" || key == "QPRO" || key == "AEXT") {
      const double t = val(0), y = val(1) * (key == "PPRO" ? 1.01325e6 : 1.0);
      if (!ok) return fail(CKMI_ERR_ARG, "bad profile line '" + line + "'");
      Profile* p = nullptr;
      for (auto& q : g_r.prof)
        if (q.key == key) p = &q;
      if (!p) {
        g_r.prof.push_back(Profile{key, {}, {}});
        p = &g_r.prof.back();
      }
      p->x.push_back(t);
      p->y.push_back(y);
    } else {
      std::string rest;
      for (size_t j = 0; j < v.size(); ++j) rest += (j ? " " : "") + v[j];
      g_r.kw.push_back({key, rest});
    }
    if (!ok) return fail(CKMI_ERR_ARG, "bad value in keyword line '" + line + "'");
  }
  if (have_x) {  // REAC mole fractions, normalised, -> mass fractions
    double sx = 0.0, sxw = 0.0;
    for (int k = 0; k < s->KK; ++k) sx += X[k];
    for (int k = 0; k < s->KK; ++k) sxw += X[k] / sx * s->wt[k];
    for (int k = 0; k < s->KK; ++k) g_r.Y0[k] = X[k] / sx * s->wt[k] / sxw;
  }
  if (!(g_r.t_end > 0.0) || !(g_r.T0 > 0.0) || !(g_r.P0 > 0.0))
    return fail(CKMI_ERR_ARG, "TIME, TEMP and PRES must be given and > 0");
  double sy = 0.0;
  for (double y : g_r.Y0) sy += y;
  if (!(sy > 0.0)) return fail(CKMI_ERR_ARG, "no initial composition (REAC)");
  g_r.done = false;
  return run_reactor(s);
}

// ---------------------------------------------------------------- declared, out of scope
// The reference declares these at import (chemkin_wrapper.py:300-867), so a drop-in library must
// export them; they belong to models outside the batch-reactor path (transport, equilibrium, PSR,
// PFR, engines, flames) and return CKMI_ERR_UNSUPPORTED with a message.
#define CKMI_OUT_OF_SCOPE(name, what, ...) \
  int name(__VA_ARGS__) { return fail(CKMI_ERR_UNSUPPORTED, #name ": " what " is not on this path"); }
CKMI_OUT_OF_SCOPE(KINGetDiffusionCoeffs, "transport", int*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINGetMixtureDiffusionCoeffs, "transport", int*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINGetOrdinaryDiffusionCoeffs, "transport", int*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINGetThermalDiffusionCoeffs, "transport", int*, double*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINCalculateEquil, "the equilibrium solver", int*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINCalculateEquilWithOption, "the equilibrium solver", int*, int*, double*, double*, double*,
                  double*)
CKMI_OUT_OF_SCOPE(KINCalculateEqGasWithOption, "the equilibrium solver", int*, int*, int*, double*, double*,
                  double*, double*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_SetupPSRReactorInputs, "the PSR model", int*, int*, double*, double*, double*, double*,
                  double*, double*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_SetupPSRInletInputs, "the PSR model", int*, int*, int*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_SetupHCCIZoneInputs, "the HCCI engine model", int*, int*, double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_SetupSIInputs, "the SI engine model", int*, double*, double*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_GetHeatRelease, "QRGEQ heat-release output", double*, double*)
CKMI_OUT_OF_SCOPE(KINAll0D_GetExitMassFlowRate, "open-reactor output", double*)
CKMI_OUT_OF_SCOPE(KINPremix_SetParameter, "the premixed flame model", char*, double*)
CKMI_OUT_OF_SCOPE(KINPremix_CalculateFlame, "the premixed flame model", int*, int*, double*, double*, double*,
                  double*, double*)
CKMI_OUT_OF_SCOPE(KINPremix_GetSolution, "the premixed flame model", int*, int*, double*, double*, double*)
CKMI_OUT_OF_SCOPE(KINPremix_GetSolutionGridPoints, "the premixed flame model", int*)
CKMI_OUT_OF_SCOPE(KINPremix_GetFlameMassFlux, "the premixed flame model", double*)
CKMI_OUT_OF_SCOPE(KINOppdif_SetInlet, "the opposed-flow flame model", char*, int*, double*, double*, double*, int*)
CKMI_OUT_OF_SCOPE(KINOppdif_SetParameter, "the opposed-flow flame model", char*, double*)
CKMI_OUT_OF_SCOPE(KINOppdif_CalculateFlame, "the opposed-flow flame model", int*, int*, double*, double*)
CKMI_OUT_OF_SCOPE(KINOppdif_GetSolutionGridPoints, "the opposed-flow flame model", int*)
CKMI_OUT_OF_SCOPE(KINOppdif_GetSolution, "the opposed-flow flame model", int*, int*, double*, double*, double**)
CKMI_OUT_OF_SCOPE(KINOppdif_GetSolnSpeciesIntegratedROP, "the opposed-flow flame model", int*, int*, int*, int*,
                  double**)
#undef CKMI_OUT_OF_SCOPE

}  // extern "C"
