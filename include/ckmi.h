/* ckmi.h -- C ABI of libckmi.so, the MI355X (gfx950) batched batch-reactor engine.
 *
 * This is the drop-in boundary for PyChemkin's batch-reactor hot path.  The reference
 * reaches the closed Chemkin library through ctypes (chemkin_wrapper.py:244,271-272) with
 * Fortran-style by-pointer scalars, caller-allocated arrays and an int error return
 * (0 = success).  libckmi keeps that convention and adds batched entry points that take
 * device-resident struct-of-arrays buffers:
 *
 *   ckmi_mech_create        replaces KINPreProcess + KINGetChemistrySizes + table getters
 *                           (chemkin_wrapper.py:303-316,333-397; chemistry.py:675-703).
 *                           The Chemkin-format text is parsed on the host
 *                           (pychemkin_amd/mechanism.py) and handed over as flat tables.
 *   ckmi_rop_thermo         batched KINGetGasROP + KINGetGasMixtureSpecificHeat /
 *                           KINGetGasMixtureEnthalpy (chemkin_wrapper.py:427-440,482-489;
 *                           mixture.py:1236,1341,1442).
 *   ckmi_reaction_rates     batched KINGetGasReactionRates (chemkin_wrapper.py:490-498;
 *                           mixture.py:1551).
 *   ckmi_species_thermo     batched KINGetGasSpecificHeat / SpeciesEnthalpy /
 *                           SpeciesInternalEnergy (chemkin_wrapper.py:375-392).
 *   ckmi_reactor_run        batched KINAll0D_SetupBatchInputs + KINAll0D_SetUserKeyword +
 *                           KINAll0D_Calculate + KINAll0D_GetIgnitionDelay +
 *                           KINAll0D_GetGasSolnResponse (chemkin_wrapper.py:606-618,
 *                           688-689,698-699,751-763; batchreactor.py:1036-1159,582,1396).
 *   ckmi_set_afactor /      KINSetAFactorForAReaction / KINGetReactionRateParameters
 *   ckmi_get_arrhenius      (chemkin_wrapper.py:499-511; chemistry.py:1627,1665).
 *
 * All buffers passed to ckmi_rop_thermo / ckmi_reaction_rates / ckmi_species_thermo /
 * ckmi_reactor_run are device pointers on the handle's device; `stream` is a hipStream_t
 * (NULL = default stream).  The calls are asynchronous on that stream.
 */
#ifndef CKMI_H
#define CKMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version returned by ckmi_version(): bumped whenever a struct layout or a table stride changes.
 * 1: round-1/2 layout (CKMI_SLOTS 4, ckmi_reactor_cfg up to prof3_v); 2: CKMI_SLOTS 8, cfg.eng[20], cfg.tran;
 * 3: desc.MM / desc.ncf (element counts) and cfg.no_elem_proj. */
#define CKMI_ABI_VERSION 3

/* the reactor kernels hold element conservation (ckmi_reactor_cfg.no_elem_proj) for mechanisms whose
 * species contain at most this many distinct elements */
#define CKMI_PROJ_MMAX 8

#define CKMI_SLOTS 8 /* distinct species per reaction side in the flat tables ([II][CKMI_SLOTS] arrays) */

/* reaction types */
#define CKMI_RXN_ELEMENTARY 0
#define CKMI_RXN_THIRDBODY 1
#define CKMI_RXN_FALLOFF 2
#define CKMI_RXN_PLOG 3 /* elementary with a PLOG table: ln k linear in ln P, clamped outside */
#define CKMI_RXN_CHEMACT 4 /* chemically activated: arr = k0, low = HIGH (k_inf); k = k0 F / (1 + Pr) */
/* Chebyshev (TCHEB / PCHEB / CHEB on a (+M) reaction): log10 k = sum_t sum_p a[t][p] T_t(Tr) T_p(Pr),
 * Tr = (2/T - 1/Tmin - 1/Tmax) / (1/Tmax - 1/Tmin), Pr = (2 log P - log Pmin - log Pmax) /
 * (log Pmax - log Pmin), no [M] factor, not clamped outside the range.  Its plog_par rows:
 * (NT, NP, 0, 0), (Tmin [K], Tmax [K], Pmin [atm], Pmax [atm]), then a[t][p] t-major, 4 per row. */
#define CKMI_RXN_CHEB 5
/* Landau-Teller elementary reaction: k = A T^b exp(-E/RT + B T^(-1/3) + C T^(-2/3)), low = (B, C, 0);
 * with REV, fpar[0..1] = the RLT (B, C) of the reverse rate */
#define CKMI_RXN_LT 6
/* falloff forms */
#define CKMI_FALL_NONE 0
#define CKMI_FALL_LINDEMANN 1
#define CKMI_FALL_TROE3 2
#define CKMI_FALL_TROE4 3
#define CKMI_FALL_SRI 4

/* error codes (0 = success, as the KIN* functions) */
#define CKMI_OK 0
#define CKMI_ERR_ARG 1
#define CKMI_ERR_HIP 2
#define CKMI_ERR_SIZE 3
#define CKMI_ERR_UNSUPPORTED 4

/* Flat mechanism tables (host pointers), layout produced by Mechanism.to_tables(). */
typedef struct {
  int32_t KK, II;
  const double* wt;       /* [KK] molecular weights, g/mol */
  const double* thermo;   /* [KK][17]: tlow, tmid, thigh, low a1..a7, high a1..a7 */
  const int32_t* rtype;   /* [II] CKMI_RXN_* */
  const int32_t* rev;     /* [II] 1 reversible */
  const int32_t* nr;      /* [II] reactant slots used */
  const int32_t* np;      /* [II] product slots used */
  const int32_t* rsp;     /* [II][CKMI_SLOTS] reactant species */
  const int32_t* psp;     /* [II][CKMI_SLOTS] product species */
  const double* rnu;      /* [II][CKMI_SLOTS] reactant stoichiometric coefficients */
  const double* pnu;      /* [II][CKMI_SLOTS] product stoichiometric coefficients */
  const double* arr;      /* [II][3] ln A (cgs), b, E/R (K) */
  const double* low;      /* [II][3] falloff low-pressure limit */
  const double* revp;     /* [II][3] explicit reverse parameters (REV) */
  const int32_t* has_rev; /* [II] */
  const int32_t* ftype;   /* [II] CKMI_FALL_* */
  const double* fpar;     /* [II][5] TROE a,T***,T*,T** or SRI a,b,c,d,e */
  const int32_t* tbsp;    /* [II] -1 mixture M, else collider species index */
  const int32_t* eff_ptr; /* [II+1] CSR into eff_sp / eff_val */
  const int32_t* eff_sp;
  const double* eff_val;  /* third-body efficiencies (absolute) */
  const int32_t* plog_ptr; /* [II+1] CSR into plog_par for CKMI_RXN_PLOG reactions (may be NULL if none) */
  const double* plog_par;  /* [npl][4] ln P (dyn/cm2), ln A (cgs), b, E/R (K); ascending, distinct P */
  const double* ford;      /* [II][CKMI_SLOTS] forward order of each reactant slot (FORD; = rnu without it), or NULL */
  const double* rord;      /* [II][CKMI_SLOTS] reverse order of each product slot (RORD; = pnu without it), or NULL */
  int32_t MM;              /* elements (0 with ncf NULL: the reactors do not hold element conservation) */
  const int32_t* ncf;      /* [MM][KK] element counts of each species (KINGetGasSpeciesComposition), or NULL */
} ckmi_mech_desc;

typedef struct ckmi_mech ckmi_mech; /* opaque: tables resident in HBM of one device */

/* Reactor-run configuration (one per batch; the reference passes these as keyword text,
 * reactormodel.py:966-996, batchreactor.py:1106-1114). */
typedef struct {
  int32_t energy;      /* 1 ENERGY equation, 2 given (constant) temperature */
  double t_end;        /* TIME [s] */
  double atol, rtol;   /* ATOL / RTOL */
  double h0;           /* HO initial step [s], 0 = estimate */
  double hmax;         /* STPT max step [s], 0 = t_end/100 */
  int32_t nneg;        /* NNEG */
  int32_t ign_mode;    /* 0 none, 1 TIFP, 2 DTIGN, 3 TLIM, 4 KLIM */
  double ign_val;      /* DTIGN rise [K] or TLIM temperature [K] */
  int32_t ign_species; /* KLIM species index */
  int32_t ign_stop;    /* IGN_STOP */
  int32_t max_steps;   /* 0 = 200000 */
  int32_t nprof;       /* VPRO (CONV) / PPRO (CONP) / TPRO profile points, 0 = none (<= 64) */
  double prof_t[64];
  double prof_v[64];
  int32_t prof_kind;   /* 0: the profile is VPRO (CONV) or PPRO (CONP); 1: TPRO (energy = 2) */
  double gfac;         /* GFAC gas-phase rate multiplier (reactormodel.py:1452-1468); 0 is read as 1 */
  double qloss;        /* QLOS heat loss rate to the surroundings [cal/s] (batchreactor.py:1884-1907) */
  double htc;          /* HTC wall heat-transfer coefficient [cal/cm2-K-s] (:1910-1939) */
  double areaq;        /* AREAQ heat-transfer area [cm2] (:1974-2003) */
  double tamb;         /* TAMB ambient temperature [K] (:1942-1971) */
  int32_t asteps;      /* ADAP/ASTEPS: extra solution point every asteps steps, 0 = off (:373-460) */
  int32_t avar;        /* ADAP/AVAR: extra point when variable avar changed by avalue since the last
                          one; -1 off, 0 temperature, 1 + k mass fraction of species k */
  double avalue;       /* AVALUE */
  int32_t nprof2;      /* second profile (energy runs), 0 = none (<= 64): */
  int32_t prof2_kind;  /* 1 QPRO heat loss rate [cal/s] (replaces QLOS), 2 AEXT area [cm2] (replaces AREAQ) */
  double prof2_t[64];
  double prof2_v[64];
  int32_t nprof3;      /* AEXT area profile [cm2] beside a QPRO in the second slot (prof2_kind 1): the */
  double prof3_t[64];  /* heat loss is then QPRO(t) + HTC AEXT(t) (T - TAMB) (batchreactor.py:2005-2067); */
  double prof3_v[64];  /* 0 = none (<= 64) */
  /* problem 4 (single-zone IC engine, KINAll0D_SetupHCCIInputs, engines/HCCI.py): CKMI_ENG_* parameters */
  double eng[20];
  /* [KK][8] device: ln-T cubics of ln eta_k [g/(cm s)] (0..3, ckmi_transport_fit) and ln lambda_k
   * [erg/(cm s K)] (4..7, ckmi_conductivity_fit) for the engine's ICHX wall heat transfer (else NULL) */
  const double* tran;
  /* 0 (default): element conservation is held to 0.1 rtol -- after an accepted step whose element content
   * (sum_k a_mk Y_k / W_k) has drifted by more than 0.1 rtol of the largest element content from the
   * initial mixture's, the corrector is projected back onto it (oracle/ckoracle.c elem_project);
   * 1: no projection (diagnostics) */
  int32_t no_elem_proj;
} ckmi_reactor_cfg;

/* engine parameter block (ckmi_reactor_cfg.eng; oracle/ckoracle.h CKO_ENG_* is the same layout) */
#define CKMI_ENG_CA0 0      /* DEG0 crank angle at t = 0 [deg] */
#define CKMI_ENG_RPM 1      /* RPM */
#define CKMI_ENG_CMPR 2     /* CMPR compression ratio */
#define CKMI_ENG_BORE 3     /* BORE [cm] */
#define CKMI_ENG_STROKE 4   /* STRK [cm] */
#define CKMI_ENG_LOLR 5     /* connecting rod length / crank radius */
#define CKMI_ENG_POLEN 6    /* POLEN piston pin offset [cm] */
#define CKMI_ENG_HTMODEL 7  /* 0 adiabatic, 1 ICHX (Nu = a Re^b Pr^c, tran required) */
#define CKMI_ENG_HTA 8
#define CKMI_ENG_HTB 9
#define CKMI_ENG_HTC 10
#define CKMI_ENG_TWALL 11   /* [K] */
#define CKMI_ENG_C11 12     /* GVEL Woschni C11 C12 C2 swirl ratio */
#define CKMI_ENG_C12 13
#define CKMI_ENG_C2 14
#define CKMI_ENG_SWIRL 15
#define CKMI_ENG_CYBAR 16   /* cylinder-head (clearance) surface / bore area */
#define CKMI_ENG_PSBAR 17   /* piston-head surface / bore area */

/* Optional per-reactor inputs / outputs of ckmi_reactor_run_ex (any pointer may be NULL). */
typedef struct {
  /* brute-force A-factor sensitivity (sensitivity.py:141-160, chemistry.py:1636-1678): reactor r
   * runs with the pre-exponential factor of reaction afac_rxn[r] (0-based, original order;
   * < 0 = none) multiplied by afac[r]. */
  const int32_t* afac_rxn; /* [n] device */
  const double* afac;      /* [n] device */
  /* adaptive solution points (cfg.asteps > 0): up to max_adap per reactor */
  int32_t max_adap;
  double* t_adap;          /* [n][max_adap] device */
  double* y_adap;          /* [n][max_adap][KK+1] device (T, Y) */
  int32_t* n_adap;         /* [n] device: points written */
  /* time of the final state (Tend, Yend): t_end, or the time the run stopped early (IGN_STOP,
   * solver failure).  DTSV rows after it (y_save) are NaN. */
  double* t_stop;          /* [n] device */
} ckmi_reactor_ext;

/* per-reactor statistics written by ckmi_reactor_run (int32 [n][8]) */
#define CKMI_STAT_NST 0
#define CKMI_STAT_NFE 1
#define CKMI_STAT_NJE 2
#define CKMI_STAT_NLU 3
#define CKMI_STAT_NCF 4
#define CKMI_STAT_NEF 5
#define CKMI_STAT_STATUS 6
#define CKMI_STAT_NNI 7 /* Newton iterations = linear solves */
#define CKMI_NSTAT 8

/* reactor status (CKMI_STAT_STATUS) */
#define CKMI_RUN_OK 0
#define CKMI_RUN_MAXSTEPS 1
#define CKMI_RUN_ERRTEST 2
#define CKMI_RUN_CONVFAIL 3
/* the state left the physical domain after an accepted step and the run was ended there: a mass
 * fraction below -max(1e-3, 1e3 atol), or (energy runs) T outside [min_k T_low,k / 2, 2 max_k T_high,k]
 * of the NASA-7 fits (the margin lets legitimately hot runs extrapolate the fits).  Without NNEG a loose tolerance can let trace concentrations go negative and
 * drive bimolecular rates of the wrong sign until the temperature runs away; the guard ends such a
 * reactor at once instead of letting it burn max_steps. */
#define CKMI_RUN_RUNAWAY 4
/* plug flow (problem 3) without a PPRO profile: the accepted state has no subsonic solution of the
 * inviscid momentum equation P + G u = P0 + G u0 any more (P0 + G u0)^2 < 4 G^2 R T / Wbar -- the
 * tube is choked (thermally, at the isothermal sound speed) and the run ends there */
#define CKMI_RUN_CHOKED 5

/* Native Chemkin-II interpreter (host only, no GPU): the parse half of KINPreProcess
 * (chemkin_wrapper.py:303-316).  chem.inp text (+ optional therm.dat text; an inline THERMO block
 * overrides it) -> the ckmi_mech_desc tables, symbols, atomic weights and element counts.  Same
 * grammar and bitwise the same tables as pychemkin_amd/mechanism.py (tests/test_parse_native.py).
 * The desc pointers stay valid until ckmi_parsed_free. */
typedef struct ckmi_parsed ckmi_parsed;
int ckmi_parse_mechanism(const char* chem_text, const char* therm_text, ckmi_parsed** out);
int ckmi_parse_files(const char* chemfile, const char* thermfile, ckmi_parsed** out);
const char* ckmi_parse_last_error(void);
void ckmi_parsed_free(ckmi_parsed* p);
int ckmi_parsed_sizes(const ckmi_parsed* p, int32_t* MM, int32_t* KK, int32_t* II);
int ckmi_parsed_desc(const ckmi_parsed* p, ckmi_mech_desc* desc);
/* species [KK][16] and elements [MM][16] NUL-padded, awt [MM], ncf [MM][KK] row-major (any may be NULL) */
int ckmi_parsed_symbols(const ckmi_parsed* p, char* species, char* elements, double* awt, int32_t* ncf);
/* reaction i (0-based) as written in the file, whitespace removed */
int ckmi_parsed_equation(const ckmi_parsed* p, int32_t i, char* buf, int32_t cap, int32_t* len);

const char* ckmi_last_error(void);
int ckmi_version(void);

/* Build device tables on the current HIP device. */
int ckmi_mech_create(const ckmi_mech_desc* desc, ckmi_mech** out);
int ckmi_mech_destroy(ckmi_mech* mech);
int ckmi_mech_sizes(const ckmi_mech* mech, int32_t* KK, int32_t* II);

/* A-factor get/set (original reaction order, 0-based); set takes effect for later calls. */
int ckmi_get_arrhenius(const ckmi_mech* mech, double* A, double* b, double* E_R);
int ckmi_set_afactor(ckmi_mech* mech, int32_t irxn, double A);

/* Species thermo per state: cp/R, h/RT, s/R  (device, [KK][n] each; any may be NULL). */
int ckmi_species_thermo(const ckmi_mech* mech, int32_t n, const double* T, double* cp_R, double* h_RT,
                        double* s_R, void* stream);

/* Batched ROP + mixture thermo at (T, P, Y):  T[n], P[n] dyn/cm2, Y[KK][n] mass fractions
 * -> wdot[KK][n] mol/cm3-s, cp[n] erg/g-K, h[n] erg/g (cp and h may be NULL). */
int ckmi_rop_thermo(const ckmi_mech* mech, int32_t n, const double* T, const double* P, const double* Y,
                    double* wdot, double* cp, double* h, void* stream);

/* Kernel selection for ckmi_rop_thermo (process-wide): 0 = automatic (the mechanism-specialised
 * kernel -- one state per lane, generated from the mechanism and compiled with hipRTC at first use
 * -- for batches of >= 16384 states when the mechanism has no PLOG / chemically activated
 * reactions, else the generic reaction-per-lane kernel), 1 = generic kernel, 2 = specialised kernel
 * (error if it is unavailable).  ckmi_rop_jit_state: 0 not compiled yet, 1 ready, -1 unavailable
 * (ckmi_last_error() then says why). */
int ckmi_set_rop_path(int32_t path);
int ckmi_rop_jit_state(const ckmi_mech* mech, int32_t* state);
/* The generated source of the specialised kernel (len = its length; copied into buf when given) and
 * a compile-only check (hipRTC, no GPU needed; code_bytes = size of the gfx950 code object). */
int ckmi_rop_jit_source(const ckmi_mech_desc* desc, char* buf, int64_t cap, int64_t* len);
int ckmi_rop_jit_compile(const ckmi_mech_desc* desc, int64_t* code_bytes);

/* Batched forward/reverse rates of progress: qf[II][n], qr[II][n] mol/cm3-s. */
int ckmi_reaction_rates(const ckmi_mech* mech, int32_t n, const double* T, const double* P, const double* Y,
                        double* qf, double* qr, void* stream);

/* Batched closed homogeneous reactors.
 *   problem[n]   1 CONP (given pressure), 2 CONV (given volume), 3 plug flow (PFR: the integration
 *                variable is the distance x [cm]; t_end / t_save / profiles / tau are in cm; V0 is the
 *                inlet velocity [cm/s] and Vend the outlet velocity; constant flow area; the pressure
 *                from the inviscid momentum equation P + rho u^2 = P0 + rho0 u0^2, or the PPRO
 *                profile in x; replaces KINAll0D_SetupPFRInputs + KINAll0D_Calculate,
 *                chemkin_wrapper.py / flowreactors/PFR.py:498-512.  Wall heat-loss fields are not
 *                applied to plug-flow reactors; the front ends reject them.),
 *                4 single-zone IC engine (closed, V(t) from the slider-crank of cfg->eng, V0 ignored;
 *                ICHX / Woschni wall heat transfer replaces QLOS / HTC; KK + 1 <= 64 only;
 *                replaces KINAll0D_SetupHCCIInputs + KINAll0D_Calculate, engines/HCCI.py:1105-1239)
 *   T0, P0, V0   [n] initial temperature [K], pressure [dyn/cm2], volume [cm3]
 *   Y0           [n][KK] initial mass fractions (reactor-major)
 *   tau          [n] ignition delay [s] (-1 if not detected)
 *   Tend, Pend, Vend [n], Yend [n][KK] final state (at t_end, or at the stop time)
 *   stats        [n][CKMI_NSTAT] int32
 *   nsave, t_save[nsave] (device) and y_save [n][nsave][KK+1] (T, Y) optional (nsave = 0)
 */
int ckmi_reactor_run(const ckmi_mech* mech, const ckmi_reactor_cfg* cfg, int32_t n, const int32_t* problem,
                     const double* T0, const double* P0, const double* V0, const double* Y0, double* tau,
                     double* Tend, double* Pend, double* Vend, double* Yend, int32_t* stats, int32_t nsave,
                     const double* t_save, double* y_save, void* stream);

/* ckmi_reactor_run plus the optional per-reactor inputs / outputs of `ext` (NULL = none):
 * the batched form of the reference's A-factor sensitivity loop and of adaptive saving. */
int ckmi_reactor_run_ex(const ckmi_mech* mech, const ckmi_reactor_cfg* cfg, int32_t n, const int32_t* problem,
                        const double* T0, const double* P0, const double* V0, const double* Y0,
                        const ckmi_reactor_ext* ext, double* tau, double* Tend, double* Pend, double* Vend,
                        double* Yend, int32_t* stats, int32_t nsave, const double* t_save, double* y_save,
                        void* stream);

/* Heat rates of a single-zone engine run (problem 4) on its saved states, evaluated with the
 * integrator's own right-hand side: the output side of KINAll0D_GetEngineHeatRelease
 * (engine.py:953-988).  T0, P0 and Y0 [KK] (device) are the cylinder's initial state (they fix its
 * mass and the Woschni reference state); t [n] and y [n][KK+1] (T, Y; device) the saved states.
 *   ahrr[n]   apparent heat-release rate m c_v dT/dt + P dV/dt [erg/s] (chemical heat release net of
 *             the wall loss)
 *   qloss[n]  wall heat-loss rate h A (T - T_wall) [erg/s] (0 for an adiabatic engine)
 * Divide by 6 RPM for the rates per crank-angle degree. */
int ckmi_engine_heat_rates(const ckmi_mech* mech, const ckmi_reactor_cfg* cfg, double T0, double P0,
                           const double* Y0, int32_t n, const double* t, const double* y, double* ahrr,
                           double* qloss, void* stream);

/* Reactor kernel selection (diagnostic / testing): 0 = automatic (one wave per reactor for KK + 1 <= 64,
 * its Newton inverse stored in FP32 unless rtol < 1e-9; one 4-wave workgroup per reactor above, up to
 * KK + 1 = 192), 1 = the workgroup-per-reactor kernel for every mechanism (lets tests run both
 * integrators on the same GRI-3.0 reactors), 2 / 3 = the wave kernel with the FP64 / FP32-stored
 * Newton inverse whatever the tolerances.  Process-wide. */
int ckmi_set_reactor_path(int32_t path);

/* Host-only capacity query of the workgroup-per-reactor kernel (no GPU needed): the largest mechanism
 * image in bytes (MechImage, staged in LDS) it accepts for nvar = KK + 1 state variables, KKp padded
 * species and G third-body groups on a CU with lds_max bytes of LDS; -1 if none fits.  A mechanism
 * whose image is larger gets CKMI_ERR_SIZE from ckmi_reactor_run. */
int ckmi_big_max_image_bytes(int32_t nvar, int32_t KKp, int32_t G, int32_t lds_max);

/* Batched dense LU of Newton iteration matrices too large for one wave (mechanisms with more
 * than 63 species).  Replaces the factorisation inside the reference's
 * KINAll0D_Calculate (batchreactor.py:1158), which has no public entry point of its own.
 *   A     [nsys][n][n] row-major FP64 (device), overwritten by L (unit lower) and U
 *   ipiv  [nsys][n] 0-based pivot rows, LAPACK dgetrf order (row i was swapped with ipiv[i])
 *   info  [nsys] 0, or k + 1 if U(k, k) is exactly zero (dgetrf convention)
 * One workgroup per matrix; the trailing updates run on v_mfma_f64_16x16x4_f64.  n <= 192. */
#define CKMI_LU_NMAX 192
int ckmi_lu_factor_batched(int32_t nsys, int32_t n, double* A, int32_t* ipiv, int32_t* info, void* stream);
/* B[nsys][n] <- A^-1 B from the factors of ckmi_lu_factor_batched (dgetrs, one right-hand side). */
int ckmi_lu_solve_batched(int32_t nsys, int32_t n, const double* LU, const int32_t* ipiv, double* B,
                          void* stream);
const char* ckmi_lu_last_error(void);

/* Viscosity: replaces KINGetViscosity (chemkin_wrapper.py:407-412) and
 * KINGetMixtureViscosity (:442-448), evaluated by the reference's closed library from the
 * transport file preprocessed by KINPreProcess (itran = 1, chemistry.py:636-687).
 *   ckmi_transport_fit      host only: params [KK][6] = geometry, eps/k [K], sigma [A], dipole [D],
 *                           polarizability [A^3], Zrot (TRANLIB columns) -> fits [KK][4], the
 *                           coefficients of ln eta_k [g/(cm s)] as a cubic in ln T, least squares
 *                           on 50 temperatures in [tlow, thigh]
 *   ckmi_transport_create   uploads the fits and the Wilke tables onto the mechanism's device
 *   ckmi_species_viscosity  T [n] -> eta [KK][n]                          (device pointers)
 *   ckmi_mixture_viscosity  T [n], Y [KK][n] mass fractions -> eta [n]    (device pointers, Wilke) */
typedef struct ckmi_transport ckmi_transport;
/* fit interval of KINPreProcess (and of pychemkin_amd/transport.py) */
#define CKMI_VISC_FIT_TLOW 300.0
#define CKMI_VISC_FIT_THIGH 3500.0
int ckmi_transport_fit(int32_t KK, const double* wt, const double* params, double tlow, double thigh, double* fits);
/* Thermal conductivity fits (host only; the engine's wall heat transfer, problem 4): lambda_k
 * [erg/(cm s K)] by the Warnatz form of TRANFIT (eta_k, the self-diffusion rho D_kk / eta_k, Zrot with
 * Parker's correction, Cv from the NASA-7 thermo [KK][17] of ckmi_mech_desc) -> fits [KK][4] of
 * ln lambda_k as a cubic in ln T on the same grid as ckmi_transport_fit. */
int ckmi_conductivity_fit(int32_t KK, const double* wt, const double* params, const double* thermo, double tlow,
                          double thigh, double* fits);
int ckmi_transport_create(const ckmi_mech* mech, const double* fits, ckmi_transport** out);
/* Thermal conductivity: replaces KINGetConductivity (chemkin_wrapper.py:413-418, mixture.py:1885-1909,
 * chemistry.py:1361-1396) and KINGetMixtureConductivity (:449-455, mixture.py:1979-2013).
 *   ckmi_transport_set_conductivity  uploads ckmi_conductivity_fit's [KK][4] fits beside the viscosity tables
 *   ckmi_species_conductivity        T [n] -> lambda [KK][n] erg/(cm s K)                  (device pointers)
 *   ckmi_mixture_conductivity        T [n], Y [KK][n] mass fractions -> lambda [n], mixture-averaged
 *                                    (sum X lambda + 1 / sum X / lambda) / 2                 (device pointers) */
int ckmi_transport_set_conductivity(ckmi_transport* tr, const double* cfits);
int ckmi_species_conductivity(const ckmi_transport* tr, int32_t n, const double* T, double* cond, void* stream);
int ckmi_mixture_conductivity(const ckmi_transport* tr, int32_t n, const double* T, const double* Y, double* cond,
                              void* stream);
int ckmi_transport_destroy(ckmi_transport* tr);
int ckmi_transport_fits(const ckmi_transport* tr, double* fits);
int ckmi_species_viscosity(const ckmi_transport* tr, int32_t n, const double* T, double* visc, void* stream);
int ckmi_mixture_viscosity(const ckmi_transport* tr, int32_t n, const double* T, const double* Y, double* visc,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif
