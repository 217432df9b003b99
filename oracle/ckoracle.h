/* ckoracle.h -- CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the batch-reactor hot path that the reference delegates to the
 * closed Chemkin library: NASA-7 thermo (KINGetGasSpecificHeat / SpeciesEnthalpy,
 * chemkin_wrapper.py:375-392), rate of production (KINGetGasROP / KINGetGasReactionRates,
 * chemkin_wrapper.py:482-498, called from mixture.py:1442,1551) and the closed-homogeneous
 * batch reactor integration (KINAll0D_Calculate, batchreactor.py:1149-1159) with ignition
 * detection (KINAll0D_GetIgnitionDelay, batchreactor.py:582) and DTSV solution saving
 * (KINAll0D_GetGasSolnResponse, batchreactor.py:1396).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product (pychemkin_amd / libckmi.so) never links or calls it.
 */
#ifndef CKORACLE_H
#define CKORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define CKO_SLOTS 8 /* = CKMI_SLOTS: distinct species per reaction side */

typedef struct {
  int KK, II;
  const double* wt;      /* [KK] g/mol */
  const double* thermo;  /* [KK][17]: tlow, tmid, thigh, low a1..a7, high a1..a7 */
  const int* rtype;      /* 0 elementary, 1 third body, 2 falloff, 3 PLOG, 4 chemically activated */
  const int* rev;        /* reversible flag */
  const int* nr; const int* np;
  const int* rsp; const int* psp;      /* [II][4] */
  const double* rnu; const double* pnu;/* [II][4] */
  const double* arr;     /* [II][3] lnA, b, E/R */
  const double* low;     /* [II][3] */
  const double* revp;    /* [II][3] */
  const int* has_rev;
  const int* ftype;      /* 0 none, 1 Lindemann, 2 Troe3, 3 Troe4, 4 SRI */
  const double* fpar;    /* [II][5] */
  const int* tbsp;       /* -1 mixture, else species index */
  const int* eff_ptr; const int* eff_sp; const double* eff_val;
  const int* plog_ptr;   /* [II+1] CSR into plog_par (rtype 3) */
  const double* plog_par;/* [npl][4]: ln P (dyn/cm2), ln A (cgs), b, E/R; ascending P per reaction */
  const double* ford;    /* [II][4] forward order of each reactant slot (FORD; = rnu without it), or NULL */
  const double* rord;    /* [II][4] reverse order of each product slot (RORD; = pnu without it), or NULL */
  int MM;                /* elements (element projection of the corrector; 0 or > CKO_PROJ_MMAX: none) */
  const int* ncf;        /* [MM][KK] element counts of each species, or NULL */
} cko_mech;

#define CKO_PROJ_MMAX 8 /* elements the corrector's element projection handles (= CKMI_PROJ_MMAX) */

typedef struct {
  int problem;      /* 1 CONP, 2 CONV */
  int energy;       /* 1 energy equation, 2 given temperature */
  double t_end;
  double atol, rtol;
  double h0;        /* initial step, 0 = estimate */
  double hmax;      /* 0 = t_end/100 */
  int nneg;         /* clip negative mass fractions inside the RHS */
  int ign_mode;     /* 0 none, 1 TIFP, 2 DTIGN, 3 TLIM, 4 KLIM */
  double ign_val;
  int ign_species;
  int ign_stop;
  int max_steps;
  int nprof;        /* volume (CONV) or pressure (CONP) profile points, 0 = none */
  const double* prof_t;
  const double* prof_v;
  int prof_kind;    /* 0 VPRO/PPRO, 1 TPRO (energy = 2): T(t) given by the profile */
  double gfac;      /* GFAC: all gas rates x gfac */
  double qloss;     /* QLOS [cal/s] */
  double htc;       /* HTC [cal/cm2-K-s] */
  double areaq;     /* AREAQ [cm2] */
  double tamb;      /* TAMB [K] */
  int pert_rxn;     /* reaction whose A factor is multiplied by pert_fac (-1 none) */
  double pert_fac;
  int nprof2;       /* second profile: QPRO [cal/s] (prof2_kind 1) or AEXT [cm2] (2), energy runs */
  int prof2_kind;
  const double* prof2_t;
  const double* prof2_v;
  int nprof3;       /* AEXT [cm2] beside a QPRO second profile (prof2_kind 1), 0 = none */
  const double* prof3_t;
  const double* prof3_v;
  const double* eng;  /* problem 4 (single-zone IC engine): CKO_ENG_N parameters, CKO_ENG_* layout */
  const double* tran; /* [KK][8]: cubic ln-T fits of ln viscosity [g/cm-s] (0..3) and ln conductivity
                         [erg/cm-K-s] (4..7), for the engine's wall heat transfer (NULL: none) */
  int no_elem_proj;   /* 1: no element projection of the accepted corrector (A/B and diagnostics only) */
} cko_cfg;

/* engine parameter block (problem 4; same layout as ckmi_reactor_cfg.eng, include/ckmi.h) */
enum {
  CKO_ENG_CA0 = 0,   /* DEG0 crank angle at t = 0 [deg] */
  CKO_ENG_RPM,       /* RPM */
  CKO_ENG_CMPR,      /* CMPR compression ratio */
  CKO_ENG_BORE,      /* BORE [cm] */
  CKO_ENG_STROKE,    /* STRK [cm] */
  CKO_ENG_LOLR,      /* connecting rod length / crank radius */
  CKO_ENG_POLEN,     /* POLEN piston pin offset [cm] */
  CKO_ENG_HTMODEL,   /* 0 adiabatic, 1 ICHX: Nu = a Re^b Pr^c */
  CKO_ENG_HTA, CKO_ENG_HTB, CKO_ENG_HTC, CKO_ENG_TWALL,
  CKO_ENG_C11, CKO_ENG_C12, CKO_ENG_C2, CKO_ENG_SWIRL, /* GVEL Woschni gas velocity */
  CKO_ENG_CYBAR, CKO_ENG_PSBAR, /* cylinder-head / piston-head area over the bore area */
  CKO_ENG_N = 20    /* 18, 19 reserved (0) */
};

typedef struct {
  double tau;       /* ignition delay [s], -1 if not detected */
  double t_end, T, P, V;
  int status;       /* 0 ok, 1 max steps, 2 error-test failures, 3 convergence failures, 4 bad state */
  int nst, nfe, nje, nlu, ncf, nef;
} cko_result;

/* thermo: per-species cp/R, h/RT, s/R at T */
void cko_thermo(const cko_mech* m, double T, double* cp_R, double* h_RT, double* s_R);
/* forward / reverse progress rates [mol/cm3-s] and species production [mol/cm3-s] at (T, P, Y) */
void cko_rates(const cko_mech* m, double T, double P, const double* Y, double* qf, double* qr, double* wdot);
/* batch of states: wdot[n][KK], cp_mass[n] [erg/g-K], h_mass[n] [erg/g] */
void cko_rop_batch(const cko_mech* m, int n, const double* T, const double* P, const double* Y,
                   double* wdot, double* cp, double* h, int nthreads);
/* one reactor; trajectory at nsave times (t_save[]) into y_save[nsave][KK+1] (T, Y), P_save, V_save */
int cko_reactor(const cko_mech* m, const cko_cfg* cfg, double T0, double P0, double V0, const double* Y0,
                double* Yend, cko_result* res, int nsave, const double* t_save, double* y_save,
                double* p_save, double* v_save);
/* batch of independent reactors with per-reactor problem type; OpenMP over reactors */
int cko_reactor_batch(const cko_mech* m, const cko_cfg* cfg, int n, const int* problem, const double* T0,
                      const double* P0, const double* V0, const double* Y0, double* Yend,
                      cko_result* res, int nthreads);
/* batch with a per-reactor A-factor perturbation (brute-force sensitivity) */
int cko_reactor_batch_pert(const cko_mech* m, const cko_cfg* cfg, int n, const int* problem, const double* T0,
                           const double* P0, const double* V0, const double* Y0, const int* pert_rxn,
                           const double* pert_fac, double* Yend, cko_result* res, int nthreads);
/* dense analytic Jacobian of the batch-reactor RHS (for tests) */
void cko_rhs_jac(const cko_mech* m, const cko_cfg* cfg, double t, const double* y, double mass_density0,
                 double V0, double P0, double* f, double* J);

#ifdef __cplusplus
}
#endif
#endif
