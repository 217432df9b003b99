/* ckmi_kin.h -- KIN-compatible C ABI of libckmi.so (drop-in for the reference's ctypes binding).
 *
 * PyChemkin binds the closed libKINetics.so with ctypes (chemkin_wrapper.py:244,271-272): scalars
 * by pointer, caller-allocated HOST arrays (np.ctypeslib.ndpointer), int return (0 = success),
 * one configured 0-D reactor per process.  libckmi.so exports all 86 symbols the reference declares
 * at import (chemkin_wrapper.py:300-867), with exactly those prototypes (line of each cited), so
 * chemkin_wrapper.py binds it unchanged.  The batch-reactor path -- KINPreProcess (native
 * Chemkin-II interpreter, ckmi_parse.cpp), sizes / symbols / weights, thermo, density, ROP, rates,
 * A-factors, the real-gas status queries (ideal gas), the 0-D batch reactor in API and full-keyword
 * mode -- is implemented on the gfx950 kernels (a batch of one state or one reactor; the batched
 * ckmi_* entry points of ckmi.h remain the fast path for sweeps).  The symbols of other models
 * (transport, equilibrium, PSR, PFR, engines, flames) return CKMI_ERR_UNSUPPORTED with a message.
 *
 * ckmi_kin_register is an extra entry point: it registers tables parsed elsewhere (the package's
 * Python interpreter, pychemkin_amd/mechanism.py) as a chemistry set.
 *
 * Units are cgs (KINSetUnitSystem(1), __init__.py:106-107); species properties from the
 * KINGetGas* thermo calls are per mass (erg/g, erg/g-K), as the reference expects
 * (chemistry.py:1127,1233,1302 multiply by WT).  Calls are serialised by a process-wide mutex.
 */
#ifndef CKMI_KIN_H
#define CKMI_KIN_H

#include <stdint.h>

#include "ckmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Register flat mechanism tables as a chemistry set on the current HIP device (replaces the parse
 * step of KINPreProcess).  names: KK species symbols, 16 chars each, NUL-padded ([KK][16]);
 * elements: MM element symbols ([MM][16]); awt [MM] g/mol; ncf [MM][KK] row-major element counts.
 * Any of names / elements / awt / ncf may be NULL (MM is then 0). */
int ckmi_kin_register(const ckmi_mech_desc* desc, int32_t MM, const char* names, const char* elements,
                      const double* awt, const int32_t* ncf, int32_t* chemset);
int ckmi_kin_release(int32_t chemset);
const char* ckmi_kin_last_error(void);
/* The reactor keyword policy shared by KINAll0D_Calculate and the Python drop-in: 1 = sets a
 * ckmi_reactor_cfg field, 2 = accepted without effect on the device path, 0 = rejected. */
int ckmi_kin_keyword_class(const char* key);

/* ---- session and preprocessing (chemkin_wrapper.py:300-331) */
/* :303-316.  Parses chem (+ therm; an inline THERMO block overrides it) with the native interpreter
 * and returns the chemistry-set index.  isurf must be 0; with itran = 1 the transport file must be
 * readable; summary (if named) receives the symbol / reaction listing; link files are not written. */
int KINPreProcess(int* isurf, int* itran, char* chem, char* surf, char* therm, char* tran, char* gaslink,
                  char* surflink, char* tranlink, char* summary, int* chemset);
int KINSetUnitSystem(int* code);                               /* :300-301 (1 = cgs only) */
int KINInitialize(int* chemset, int* flag);                    /* :317-320 */
void KINFinish(void);                                          /* :321-322 */
int KINUpdateChemistrySet(int* chemset);                       /* :323-326 */
int KINSwitchChemistrySet(int* chemset);                       /* :327-331 */

/* ---- sizes and tables (:333-397) */
int KINGetChemistrySizes(int* chemset, int* MM, int* KK, int* II, int* nmat, int* nsite, int* nbulk, int* nphase,
                         int* nsurfrxn);                                        /* :333-344 */
int KINGetGasSpeciesNames(int* chemset, char** names);                          /* :345-349 */
int KINGetElementNames(int* chemset, char** names);                             /* :350-354 */
int KINGetAtomicWeights(int* chemset, double* awt);                             /* :355-359 */
int KINGetGasMolecularWeights(int* chemset, double* wt);                        /* :360-364 */
int KINGetGasSpeciesComposition(int* chemset, int32_t* ncf);                    /* :393-397, [MM,KK] F-order */
int KINGetGasReactionString(int* chemset, int* irxn, int* len, char* buf);      /* :365-371, 1-based, KINPreProcess sets */
int KINGetReactionStringLength(int* len);                                       /* :372-373, longest, active set */
int KINGetMassFractionFromMoleFraction(int* chemset, double* X, double* Y);     /* :855-860 */
int KINGetMoleFractionFromMassFraction(int* chemset, double* Y, double* X);     /* :862-867 */

/* ---- real-gas EOS (:545-581): ideal gas only.  GetEOSMode / CheckRealGasStatus answer mode 0
 * (chemistry.py:755-792, realgaseos.py:30-52 read it as "ideal gas"); UseIdealGasLaw and
 * SetCurrentPressure succeed; the cubic-EOS setters return CKMI_ERR_UNSUPPORTED. */
int KINRealGas_SetParameter(char* key, double* value);                          /* :545-549 */
int KINRealGas_GetEOSMode(int* chemset, int* mode, char* name);                 /* :550-555 */
int KINRealGas_SetMixingRule(int* chemset, int* rule, int* flag);               /* :556-561 */
int KINRealGas_UseIdealGasLaw(int* chemset, int* flag);                         /* :562-566 */
int KINRealGas_UseCubicEOS(int* chemset, int* mode);                            /* :567-571 */
int KINRealGas_SetCurrentPressure(int* chemset, double* P);                     /* :572-576 */
int KINRealGas_CheckRealGasStatus(int* chemset, int* mode);                     /* :577-581 */
int KINGetGamma(int* chemset, double* T, double* Y, double* gamma);             /* :582-588, cp / cv */

/* ---- thermo (per mass), density (:375-440) */
int KINGetGasSpecificHeat(int* chemset, double* T, double* cp);                 /* :375-380, erg/g-K [KK] */
int KINGetGasSpeciesEnthalpy(int* chemset, double* T, double* h);               /* :381-386, erg/g [KK] */
int KINGetGasSpeciesInternalEnergy(int* chemset, double* T, double* u);         /* :387-392, erg/g [KK] */
int KINGetMassDensity(int* chemset, double* T, double* P, double* Y, double* rho); /* :398-405, g/cm3 */
int KINGetGasMixtureSpecificHeat(int* chemset, double* T, double* Y, double* cp); /* :427-433, erg/g-K */
int KINGetGasMixtureEnthalpy(int* chemset, double* T, double* Y, double* h);    /* :434-440, erg/g */

/* ---- kinetics (:482-511) */
int KINGetGasROP(int* chemset, double* T, double* P, double* Y, double* wdot);  /* :482-489, mol/cm3-s [KK] */
/* :490-498.  The composition is read as MOLE fractions (Chemkin CKKFKR convention; what the closed
 * library does, as reactionrates.baseline shows -- see DESIGN.md "reaction rates golden"). */
int KINGetGasReactionRates(int* chemset, double* T, double* P, double* X, double* qf, double* qr);
int KINGetReactionRateParameters(int* chemset, double* A, double* b, double* E_R); /* :499-505 */
int KINSetAFactorForAReaction(int* chemset, int* irxn, double* A);              /* :506-511: irxn > 0 get, < 0 put */

/* ---- 0-D batch reactor (:590-763) */
int KINAll0D_Setup(int* chemset, int* reactortype, int* problem, int* energy, int* solver, int* npsr,
                   int32_t* ninlets, int* nzones);                              /* :590-600 */
int KINAll0D_SetupWorkArrays(int* lout, int* chemset);                          /* :601-605 */
int KINAll0D_SetupBatchInputs(int* chemset, double* t_end, double* T, double* P, double* V, double* qloss,
                              double* area, double* Y, double* site, double* bulk); /* :606-618 */
int KINAll0D_IntegrateHeatRelease(void);                                        /* :700-701 */
int KINAll0D_SetProfilePoints(int* npoints);                                    /* :710-711 */
int KINAll0D_SetProfileParameter(char* key, int* npoints, double* x, double* y); /* :712-718 */
int KINAll0D_SetUserKeyword(char* line);                                        /* :698-699 */
int KINAll0D_Calculate(int* chemset);                                           /* :688-689 */
int KINAll0D_GetIgnitionDelay(double* tau);                                     /* :762-763, s */
int KINAll0D_GetSolnResponseSize(int* nreac, int* npts);                        /* :746-750 */
int KINAll0D_GetGasSolnResponse(int* nreac, int* npts, int* KK, double* t, double* T, double* P, double* V,
                                double* Y);                                     /* :751-761, Y [KK,npts] F-order */
/* :690-697, the full-keyword mode (batchreactor.py:822-978): one string of nlines keyword lines of
 * lengths linelen[] (TRAN, CONP|CONV, ENRG|TGIV, PRES [atm], TEMP, TIME, REAC sp x, VOL, profile
 * points, QRGEQ, END and the API-mode keywords), then the run */
int KINAll0D_CalculateInput(int* lout, int* chemset, char* lines, int* nlines, int32_t* linelen);
/* API-mode setters declared by the reference (:702-738), each the keyword it stands for */
int KINAll0D_SetHeatTransfer(double* htc, double* tamb);                        /* :702-706, HTC + TAMB */
int KINAll0D_SetHeatTransferArea(double* area);                                 /* :707-708, AREAQ */
int KINAll0D_SetProfileKeyword(int* a, int* b, char* key, int* npoints, double* x, double* y); /* :719-727 */
int KINAll0D_SetSolverInitialStepTime(double* h0);                              /* :729-730, HO */
int KINAll0D_SetSolverMaximumStepTime(double* hmax);                            /* :731-732, STPT */
int KINAll0D_SetSolverMaximumIteration(int* n);                                 /* :733-734, MAXIT */
int KINAll0D_SetRelaxIteration(void);                                           /* :735-736, unsupported */
int KINAll0D_SetMinimumSpeciesBound(double* v);                                 /* :737-738, unsupported */
int KINAll0D_GetSolution(double* T, double* P, double* Y);                      /* :739-745, final state */

/* ---- declared by the reference for other models: CKMI_ERR_UNSUPPORTED + message */
int KINGetViscosity(int*, double*, double*);                                    /* :407-412 */
int KINGetConductivity(int*, double*, double*);                                 /* :413-418 */
int KINGetDiffusionCoeffs(int*, double*, double*, double*);                     /* :419-425 */
int KINGetMixtureViscosity(int*, double*, double*, double*);                    /* :442-447 */
int KINGetMixtureConductivity(int*, double*, double*, double*);                 /* :449-454 */
int KINGetMixtureDiffusionCoeffs(int*, double*, double*, double*, double*);     /* :456-462 */
int KINGetOrdinaryDiffusionCoeffs(int*, double*, double*, double*, double*);    /* :464-470 */
int KINGetThermalDiffusionCoeffs(int*, double*, double*, double*, double*, double*); /* :472-479 */
int KINCalculateEquil(int*, double*, double*, double*, double*);                /* :513-519 */
int KINCalculateEquilWithOption(int*, int*, double*, double*, double*, double*); /* :521-528 */
int KINCalculateEqGasWithOption(int*, int*, int*, double*, double*, double*, double*, double*, double*,
                                double*, double*);                              /* :530-543 */
int KINAll0D_SetupPSRReactorInputs(int*, int*, double*, double*, double*, double*, double*, double*, double*,
                                   double*, double*, double*);                  /* :619-632 */
int KINAll0D_SetupPSRInletInputs(int*, int*, int*, double*, double*, double*);  /* :634-641 */
int KINAll0D_SetupPFRInputs(int*, double*, double*, double*, double*, double*, double*, double*, double*,
                            double*, double*);                                  /* :643-655 */
int KINAll0D_SetupHCCIInputs(int*, double*, double*, double*, double*, double*, double*, double*, double*,
                             double*, double*, double*);                        /* :657-670 */
int KINAll0D_SetupHCCIZoneInputs(int*, int*, double*, double*);                 /* :672-677 */
int KINAll0D_SetupSIInputs(int*, double*, double*, double*, double*, double*);  /* :679-686 */
int KINAll0D_GetHeatRelease(double*, double*);                                  /* :764-768 */
int KINAll0D_GetEngineHeatRelease(double*, double*, double*, double*, double*, double*); /* :769-777 */
int KINAll0D_GetExitMassFlowRate(double*);                                      /* :778-779 */
int KINPremix_SetParameter(char*, double*);                                     /* :781-785 */
int KINPremix_CalculateFlame(int*, int*, double*, double*, double*, double*, double*); /* :786-795 */
int KINPremix_GetSolution(int*, int*, double*, double*, double*);               /* :796-803 */
int KINPremix_GetSolutionGridPoints(int*);                                      /* :804-807 */
int KINPremix_GetFlameMassFlux(double*);                                        /* :808-811 */
int KINOppdif_SetInlet(char*, int*, double*, double*, double*, int*);           /* :812,818-825 */
int KINOppdif_SetParameter(char*, double*);                                     /* :813,826-829 */
int KINOppdif_CalculateFlame(int*, int*, double*, double*);                     /* :814,830-836 */
int KINOppdif_GetSolutionGridPoints(int*);                                      /* :815,837 */
int KINOppdif_GetSolution(int*, int*, double*, double*, double**);              /* :816,838-844 */
int KINOppdif_GetSolnSpeciesIntegratedROP(int*, int*, int*, int*, double**);    /* :845-852 */

#ifdef __cplusplus
}
#endif
#endif
