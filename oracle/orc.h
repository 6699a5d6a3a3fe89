/*
 * orc.h -- CPU ORACLE for the PINC per-timestep PIC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This directory is a plain-C restatement of the
 * reference algorithm (trymen/PINC, /root/reference/src) used as the checker
 * for the MI355X path in pinc_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Pinning: the reference itself cannot be compiled here (core.h:12 includes
 * <gsl/gsl_rng.h>; GSL is absent from the image, and a reference build would
 * need stand-in headers, which this project does not write).  The oracle is
 * therefore pinned against (1) the known-answer values in the reference's own
 * unit tests (test/pusher.test.c, test/grid.test.c) and (2) the reference
 * outputs recorded in SURVEY.md Appendix B (KE/PE of step 1, Langmuir
 * frequencies, V-cycle counts).  See DESIGN.md "Oracle".
 *
 * Multi-rank runs are emulated in one process: a "world" holds one rank
 * context per subdomain and every MPI exchange of the reference becomes a
 * copy between rank contexts (same message contents, deterministic order).
 */
#ifndef ORC_H
#define ORC_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ ini -- */
/* Dictionary with iniparser-3.1 semantics: keys are "section:key",
 * lower-cased; values are raw strings (io.c:254-560, iniparser.c:555-613). */
typedef struct OIni OIni;

OIni *oini_load(const char *path);
OIni *oini_from_string(const char *text);
void oini_free(OIni *ini);
void oini_set(OIni *ini, const char *key, const char *value);
int oini_has(const OIni *ini, const char *key);
const char *oini_raw(const OIni *ini, const char *key); /* aborts if absent */
int oini_nelem(const OIni *ini, const char *key);
int oini_int(const OIni *ini, const char *key);
long oini_long(const OIni *ini, const char *key);
double oini_double(const OIni *ini, const char *key);
char **oini_strarr(const OIni *ini, const char *key, int n); /* free w/ oini_freestrarr */
void oini_freestrarr(char **arr);
int *oini_intarr(const OIni *ini, const char *key, int n);
long *oini_longarr(const OIni *ini, const char *key, int n);
double *oini_doublearr(const OIni *ini, const char *key, int n);
void oini_setdoublearr(OIni *ini, const char *key, const double *v, int n);
void oini_setdouble(OIni *ini, const char *key, double v);
void oini_scaledouble(OIni *ini, const char *key, double factor);
void oini_applysuffix(OIni *ini, const char *key, const char *suffix,
                      const double *mul, int mullen);
void orc_die(const char *fmt, ...);
/* OpenMP threads of the oracle's stencil and per-rank loops (ORC_THREADS,
 * default 1).  Only loops whose result does not depend on the visiting
 * order are parallel, so every output is bit-identical for any count. */
extern int orc_nthreads;
#define ORC_PAR_MIN 32768

/* ---------------------------------------------------------------- types -- */
typedef struct {
	int rank;          /* nDims+1 */
	int size[4];       /* [nValues, nx+2g, ny+2g, nz+2g] */
	int trueSize[4];
	long sizeProd[5];
	int nGhost[8];     /* 2*rank entries */
	double *val;
} OGrid;

typedef struct {
	int nDims, nSpecies;
	double *pos, *vel;       /* AoS, nDims doubles per particle */
	long *iStart;            /* nSpecies+1 */
	long *iStop;             /* nSpecies   */
	double *charge, *mass;
	double *kinEnergy, *potEnergy; /* nSpecies+1 */
	long *id;                /* shadow ids (oracle-only bookkeeping) */
} OPop;

typedef struct {
	int mpiRank, mpiSize, nDims, nSpecies;
	int subdomain[3], nSubdomains[3], nSubdomainsProd[4], offset[3];
	double posToSubdomain[3];
	int nNeighbors, center;
	long *nEmigrants;      /* nNeighbors*nSpecies */
	long *nEmigrantsAlloc; /* nNeighbors */
	long *nImmigrants;     /* nNeighbors*nSpecies */
	double **emigrants;    /* nNeighbors buffers, 2*nDims doubles/particle */
	long **emigrantIds;
	double thresholds[6];
} OMpi;

/* Multigrid hierarchy of one rank: grids[0] aliases the user grid. */
typedef struct {
	int nLevels;
	OGrid **grids;
} OMg;

typedef struct {
	OMpi mpi;
	OPop pop;
	OGrid E, rho, phi, res;
	OMg mgRho, mgPhi, mgRes;
} ORank;

enum { ORC_ACC_3D1KE, ORC_ACC_ND1KE, ORC_ACC_3D1, ORC_ACC_ND1, ORC_ACC_BORIS3D1KE, ORC_ACC_BORIS3D1,
       ORC_ACC_ND0KE, ORC_ACC_ND0 };
enum { ORC_DISTR_3D1, ORC_DISTR_ND1, ORC_DISTR_ND0 };
enum { ORC_MIG_3D, ORC_MIG_ND };
enum { ORC_SMOOTH_GS3D, ORC_SMOOTH_GSND };
enum { ORC_RESTR_3D, ORC_RESTR_ND };
enum { ORC_PROL_3D, ORC_PROL_ND };
enum { ORC_POISSON_MG, ORC_POISSON_SPECTRAL };

typedef struct ONative ONative;  /* orc_native.c */

typedef struct {
	int P;              /* number of subdomains (emulated ranks) */
	int nDims, nSpecies;
	ORank *r;
	OIni *ini;
	/* selected operators */
	int acc, distr, migrate, poisson;
	double borisT[24], borisS[24];  /* puGet3DRotationParameters, per species */
	int preSmooth, postSmooth, coarseSolv, restrictor, prolongator;
	int nLevels, nPre, nPost, nCoarse, mgCycles;
	double maxVel;
	/* diagnostics */
	long cycles;        /* V-cycles run so far */
	long mgCap;         /* 0: loop until converged (multigrid.c:1698); else cycles per solve */
	double *mgHist;     /* RMS residual after each cycle of the last solve */
	long mgHistCap, mgHistN;
	int verbose;        /* ORC_VERBOSE=n: MG progress every n cycles (stderr) */
	long solves;
	double lastKE, lastPE;
	double *keSpecies;  /* nSpecies */
	double weights[8];
	double unitCharge, unitMass, unitLength, unitTime;
	int literal;        /* 1: reproduce main.c double FROMHALO + 2nd solve */
	double *spectralFactor; /* 1-D spectral solver (spectral.c:29-37) */
	ONative *native;    /* multigrid:native = 1 (the device's native mode) */
	double phaseT[7];   /* ow_step wall seconds per phase */
} OWorld;

/* ---------------------------------------------------------------- grid -- */
void og_alloc(OGrid *g, const OIni *ini, int nValues);
void og_alloc_sub(OGrid *g, const OGrid *fine, int q);
void og_free(OGrid *g);
void og_zero(OGrid *g);
void og_mul(OGrid *g, double num);
void og_sub(OGrid *g, double num);
void og_addto(OGrid *res, const OGrid *add);
void og_square(OGrid *g);
double og_sum_true(const OGrid *g);
double og_pot_energy_inner(const OGrid *rho, const OGrid *phi);
void og_findiff1st(const OGrid *scalar, OGrid *field);
void og_findiff2nd(OGrid *res, const OGrid *phi);
enum { OP_SET = 0, OP_ADD = 1 };
enum { TOHALO = 0, FROMHALO = 1 };
void ow_halo(OWorld *w, OGrid **grids, int op, int dir);
void ow_halo_dim(OWorld *w, OGrid **grids, int d, int op, int dir);
void ow_neutralize(OWorld *w, OGrid **grids);
long og_tot_truesize(const OGrid *g, const OMpi *mpi);

/* ----------------------------------------------------------- population -- */
void op_alloc(OPop *p, const OIni *ini, int mpiSize);
void op_free(OPop *p);
void op_pos_lattice(OPop *p, const OIni *ini, const OMpi *mpi);
void op_pos_perturb(OPop *p, const OIni *ini, const OMpi *mpi);
void op_vel_zero(OPop *p);
void op_vel_maxwell(OPop *p, const OIni *ini, unsigned long long seed);
void op_to_local(OPop *p, const OMpi *mpi);
void op_to_global(OPop *p, const OMpi *mpi);
void op_sum_kin(OPop *p);

/* ------------------------------------------------------------- pusher -- */
void opu_move(OPop *p);
void opu_acc3d1(OPop *p, OGrid *E, int ke);
void opu_boris3d1(OPop *p, OGrid *E, const double *T, const double *S, int ke);
void opu_rotation_params(int nSpecies, const double *BExt, const double *charge, const double *mass, double *T,
                         double *S);
void opu_accnd1(OPop *p, OGrid *E, int ke);
void opu_distr3d1(const OPop *p, OGrid *rho);
void opu_distrnd1(const OPop *p, OGrid *rho);
void opu_accnd0(OPop *p, OGrid *E, int ke);
void opu_distrnd0(const OPop *p, OGrid *rho);
void opu_extract3d(OPop *p, OMpi *mpi);
void opu_extractnd(OPop *p, OMpi *mpi);
void ow_migrate(OWorld *w);
int opu_neighbor_to_rank(const OMpi *mpi, int neighbor);
int opu_rank_to_neighbor(const OMpi *mpi, int rank);
int opu_neighbor_to_reciprocal(int neighbor, int nDims);
void om_create_neighborhood(OMpi *mpi, const OIni *ini, const OGrid *g);

/* ----------------------------------------------------------- multigrid -- */
void ow_mg_alloc(OWorld *w);
void ow_mg_solve(OWorld *w);
void ow_spectral_solve(OWorld *w);
/* native-mode multigrid of the MI355X build (orc_native.c; not the
 * reference's algorithm): correction scheme with the coarse h^2 factor */
ONative *on_alloc(int nd, const int *Tglobal, int nLevelsIni, int nd3);
void on_free(ONative *S);
/* initial-guess roles (include/pinc.h PINC_MG_GUESS_*) */
#define ON_GUESS_WARM 0
#define ON_GUESS_SERIES 1
#define ON_GUESS_FIRST 2
#define ON_GUESS_SECOND 3
void on_set_extrapolate(ONative *S, int on, int objects);
void on_set_second_spectral(ONative *S, int on);
void on_set_spectral_coarse(ONative *S, int on);
void orc_discrete_poisson(int nd, const int *L, const double *rho, double *phi);
void on_guess_next(ONative *S, int role);
int on_levels(const ONative *S);
void ow_native_solve(OWorld *w);
/* single-grid stencil primitives (exported for unit tests) */
void omg_gs_pass(OGrid *phi, const OGrid *rho, int color, int nd3);
void omg_residual(OGrid *res, const OGrid *rho, const OGrid *phi);
void omg_restrict(const OGrid *fine, OGrid *coarse, int nd3);
void omg_inject(OGrid *fine, const OGrid *coarse);
void omg_prolong_dim(OGrid *fine, int r);

/* ------------------------------------------------------------ driver -- */
OWorld *ow_create(OIni *ini, int literal);
void ow_free(OWorld *w);
void ow_init(OWorld *w, int perturb, int maxwell, unsigned long long seed);
void ow_init_fields(OWorld *w);
void ow_step(OWorld *w);

/* ------------------------------------------------ immersed objects -- */
/* orc_obj.c: object.c restated for one subdomain (defects corrected, see
 * the file header) */
typedef struct OObj OObj;
OObj *oo_create(OWorld *w, const double *maskTrue);
void oo_free(OObj *o);
void oo_capacitance(OObj *o, OWorld *w);
void oo_apply(OObj *o, OWorld *w, double *phiC);
void oo_collect(OObj *o, OWorld *w);
void oo_init_collect(OObj *o, OWorld *w);
void oo_step(OWorld *w, OObj *o);
const OGrid *oo_rho_obj_grid(const OObj *o);

/* Splittable counter-based RNG shared with the product's initialiser (the
 * reference's GSL mt19937+ziggurat is absent: parity of draws is unpinned,
 * SURVEY.md 8(c)).  normal = Box-Muller on two 53-bit uniforms of
 * splitmix64(seed, counter). */
double orc_uniform(unsigned long long seed, unsigned long long counter);
double orc_normal(unsigned long long seed, unsigned long long counter);

#endif
