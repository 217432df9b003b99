/* ckmi_kin.h -- KIN-compatible C ABI of libckmi.so (drop-in for the reference's ctypes binding).
 *
 * PyChemkin binds the closed libKINetics.so with ctypes (chemkin_wrapper.py:244,271-272): scalars
 * by pointer, caller-allocated HOST arrays (np.ctypeslib.ndpointer), int return (0 = success),
 * one configured 0-D reactor per process.  These entry points keep exactly those prototypes
 * (chemkin_wrapper.py line of each is cited) so that the reference's call sites -- mixture.py,
 * chemistry.py, batchreactor.py -- run unchanged against libckmi.so.  Internally every call stages
 * host <-> device memory and runs the batched gfx950 kernels of ckmi.h (a batch of one state or one
 * reactor); the batched ckmi_* entry points remain the fast path for sweeps.
 *
 * One difference: KINPreProcess (chemkin_wrapper.py:303-316) parses chem.inp / therm.dat inside
 * the closed library.  Here the Chemkin-format parser is the host side of the package
 * (pychemkin_amd/mechanism.py, called by Chemistry.preprocess) and hands the flat tables over with
 * ckmi_kin_register, which returns the chemistry-set index every KIN* call takes.
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

/* ---- session (chemkin_wrapper.py:300-331) */
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

#ifdef __cplusplus
}
#endif
#endif
