/*
 * pinc.h -- host operator surface of the MI355X PINC hot path (libpinc.so).
 *
 * Mirrors the reference's C API so a main.c-style loop drops in unchanged
 * (reference: src/core.h, pusher.h, grid.h, population.h, multigrid.h,
 * io.h, units.h).  The structs keep the reference's fields and meaning;
 * each gains a device twin (dev*) that the operators act on.  Host arrays
 * (Population.pos/vel, Grid.val) are only refreshed by the explicit
 * *SyncToHost calls (diagnostics, parity dumps), never inside a step.
 *
 * Errors follow the reference (io.c:170-217): msg(ERROR,...) prints and
 * exits.  The PincSim API at the end returns error codes instead and is
 * what Python (bench.py, tests) drives through ctypes.
 */
#ifndef PINC_H
#define PINC_H

#ifdef __cplusplus
extern "C" {
#endif

#include "pinc_hip.h"

/* ------------------------------------------------------- core.h types -- */
typedef void (*funPtr)();
typedef struct dictionary dictionary;  /* iniparser-compatible dictionary */
typedef struct PincObj Object;        /* immersed objects (object.h:8-21) */

typedef enum { STATUS = 0x00, WARNING = 0x01, ERROR = 0x02, TIMER = 0x03, ALL = 0x10 } msgKind;
typedef enum { PERIODIC = 0x01, DIRICHLET = 0x02, NEUMANN = 0x03, NONE = 0x10 } bndType;
typedef enum { SCALAR = 1, VECTOR = -1 } gValueKind;          /* grid.h:14-17 */
typedef enum { TOHALO = 0, FROMHALO = 1 } opDirection;       /* grid.h:22-25 */

typedef struct PincDevPop PincDevPop;
typedef struct PincDevGrid PincDevGrid;

/* The structs below have the reference's fields in the reference's order,
 * types and offsets (x86-64 LP64; tests/test_core_layout.py checks every
 * offsetof against tests/golden/core_layout.json, extracted from core.h).
 * Each gains its device twin as a field appended AFTER the reference's
 * last one, so code compiled against core.h reads every reference field at
 * the offset it expects.  hid_t is HDF5 >= 1.10's int64_t (the library
 * loads HDF5 at run time); MPI_Request * is an opaque pointer slot.  Fields
 * the hot path does not use are kept NULL/0 (marked "unused"). */
typedef long long pinc_hid_t;        /* hid_t (HDF5 >= 1.10: int64_t) */

/* core.h:72-86 */
typedef struct {
	double *pos;         /* host mirror (AoS, nDims per particle)        */
	double *vel;
	long *iStart;        /* nSpecies+1 */
	long *iStop;         /* nSpecies   */
	long *objVicinity;   /* unused (NULL): object.c keeps its own lists  */
	long *collisions;    /* unused (NULL)                                 */
	double *charge;      /* normalised, nSpecies */
	double *mass;
	double *kinEnergy;   /* nSpecies+1 */
	double *potEnergy;   /* nSpecies+1 */
	int nSpecies;
	int nDims;
	pinc_hid_t h5;       /* .pop.h5 file (rank 0 only, pOpenH5) */
	PincDevPop *dev;     /* device twin (appended) */
} Population;

/* core.h:112-138 */
typedef struct {
	int mpiRank, mpiSize, nDims;
	int *subdomain, *nSubdomains, *nSubdomainsProd, *offset;
	double *posToSubdomain;
	int nSpecies, nNeighbors, neighborhoodCenter;
	long **migrants;        /* unused (NULL; DEPRECATED in the reference) */
	long **migrantsDummy;   /* unused (NULL) */
	long *nEmigrants;       /* nNeighbors*nSpecies */
	long *nEmigrantsAlloc;  /* nNeighbors */
	long *nImmigrants;      /* nNeighbors*nSpecies */
	long nImmigrantsAlloc;  /* immigrant records the device buffer holds */
	double **emigrants;     /* unused (NULL): emigrants stay on the device */
	double **emigrantsDummy;/* unused (NULL) */
	double *immigrants;     /* unused (NULL) */
	double *thresholds;     /* 2*nDims (+ nDims upper bounds for the assert) */
	void *send;             /* MPI_Request *: unused (NULL) */
	void *recv;             /* MPI_Request *: unused (NULL) */
	void *comm;             /* RCCL communicator, NULL with one rank (appended) */
} MpiInfo;

/* core.h:261-277 */
typedef struct {
	double *val;         /* host mirror, reference layout incl. ghosts */
	int rank;            /* nDims+1 */
	int *size, *trueSize;
	long *sizeProd;
	int *nGhostLayers;
	double *sendSlice;   /* unused (NULL): halos move on the device */
	double *recvSlice;   /* unused (NULL) */
	double *bndSlice;    /* unused (NULL): periodic boundaries only */
	pinc_hid_t h5;       /* .grid.h5 file (rank 0 only, gOpenH5) */
	pinc_hid_t h5MemSpace;  /* unused (0): set per write */
	pinc_hid_t h5FileSpace; /* unused (0) */
	bndType *bnd;
	PincDevGrid *dev;    /* device twin (appended) */
} Grid;

/* core.h:392-417 */
typedef struct {
	int nDims, nSpecies;
	double *weights;
	double charge, mass, length, time;
	double hyperArea, hyperVolume, frequency, velocity, acceleration, density,
	       chargeDensity, potential, eField, bField, energy;
} Units;

/* ---------------------------------------------------------------- io -- */
void msg(msgKind kind, const char *format, ...);
dictionary *iniOpen(int argc, char *argv[]);
dictionary *iniFromString(const char *text);
void iniClose(dictionary *ini);
void iniSet(dictionary *ini, const char *key, const char *value);
int iniHas(const dictionary *ini, const char *key);
int iniGetNElements(const dictionary *ini, const char *key);
int iniGetInt(const dictionary *ini, const char *key);
long iniGetLongInt(const dictionary *ini, const char *key);
double iniGetDouble(const dictionary *ini, const char *key);
char *iniGetStr(const dictionary *ini, const char *key);
int *iniGetIntArr(const dictionary *ini, const char *key, int nElements);
long *iniGetLongIntArr(const dictionary *ini, const char *key, int nElements);
double *iniGetDoubleArr(const dictionary *ini, const char *key, int nElements);
char **iniGetStrArr(const dictionary *ini, const char *key, int nElements);
void freeStrArr(char **strArr);
void iniSetDouble(dictionary *ini, const char *key, double value);
void iniSetDoubleArr(dictionary *ini, const char *key, const double *values, int nElements);
void iniScaleDouble(dictionary *ini, const char *key, double factor);
void iniApplySuffix(dictionary *ini, const char *key, const char *suffix, const double *mul, int mulLen);
/* select(ini,"methods:acc", puAcc3D1_set, ...) as io.h:105 */
funPtr selectInner(const dictionary *ini, const char *key, const char *list, ...);
/* The reference defines select() as a macro (io.h:105); include system
 * headers that declare POSIX select() before this header, or define
 * PINC_NO_SELECT_MACRO and call selectInner directly. */
#ifndef PINC_NO_SELECT_MACRO
#define select(ini, key, ...) selectInner(ini, key, #__VA_ARGS__, __VA_ARGS__)
#endif

/* --------------------------------------------------------------- aux -- */
/* Timer (core.h:439-442, aux.c:48-85): wall time in nanoseconds; tStop waits
 * for the device work queued so far, so a span measures what the reference's
 * blocking loop measured */
typedef struct {
	unsigned long long total;  /* total time */
	unsigned long long start;  /* previous start time */
} Timer;
Timer *tAlloc();        /* main.c:192 passes the rank; unused, as in aux.c */
void tFree(Timer *t);
void tStart(Timer *t);
void tStop(Timer *t);
void tReset(Timer *t);
void tMsg(long long nanoSec, const char *string);

/* ------------------------------------------------------------- units -- */
Units *uAlloc(dictionary *ini);
void uFree(Units *units);
void uNormalize(dictionary *ini, const Units *units);

/* -------------------------------------------------------------- grid -- */
Grid *gAlloc(const dictionary *ini, int nValues);
void gFree(Grid *grid);
MpiInfo *gAllocMpi(const dictionary *ini);
void gFreeMpi(MpiInfo *mpiInfo);
void gCreateNeighborhood(const dictionary *ini, MpiInfo *mpiInfo, Grid *grid);
void gDestroyNeighborhood(MpiInfo *mpiInfo);
void gSetBndSlices(Grid *grid, MpiInfo *mpiInfo);
/* slice operators are tokens selecting the halo semantics (grid.c:72-147) */
void setSlice(const double *slice, Grid *grid, int d, int offset);
void addSlice(const double *slice, Grid *grid, int d, int offset);
void gHaloOp(funPtr sliceOp, Grid *grid, const MpiInfo *mpiInfo, opDirection dir);
void gFinDiff1st(const Grid *scalar, Grid *field);
void gMul(Grid *grid, double num);
void gZero(Grid *grid);
void gAddTo(Grid *result, Grid *addition);
void gNeutralizeGrid(Grid *grid, const MpiInfo *mpiInfo);
void gPotEnergy(const Grid *rho, const Grid *phi, Population *pop);
void gSyncToHost(Grid *grid);       /* device -> reference-layout host mirror */
void gSyncToDevice(Grid *grid);     /* host mirror (true nodes) -> device */

/* -------------------------------------------------------- population -- */
Population *pAlloc(const dictionary *ini);
void pFree(Population *pop);
void pPosLattice(const dictionary *ini, Population *pop, const MpiInfo *mpiInfo);
void pPosPerturb(const dictionary *ini, Population *pop, const MpiInfo *mpiInfo);
void pVelZero(Population *pop);
void pVelMaxwell(const dictionary *ini, Population *pop, unsigned long long seed);
void pToLocalFrame(Population *pop, const MpiInfo *mpiInfo);
void pToGlobalFrame(Population *pop, const MpiInfo *mpiInfo);
void pSumKinEnergy(Population *pop);
void pSyncToHost(Population *pop);
void pSyncToDevice(Population *pop);
/* main.c:206,219 (population.c:342-365, 316-340): msg(ERROR) if a velocity
 * component exceeds max / a particle left the local frame.  The kernels that
 * move and kick the particles record both conditions in a device word; these
 * read it */
void pVelAssertMax(const Population *pop, double max);
void pPosAssertInLocalFrame(const Population *pop, const Grid *grid);
/* generate lattice (+perturbation, +Maxwellian) directly on the device */
void pInitDevice(const dictionary *ini, Population *pop, const MpiInfo *mpiInfo, int perturb,
                 int maxwell, unsigned long long seed);

/* ------------------------------------------------------------ pusher -- */
void puMove(Population *pop, Object *obj);
funPtr puAcc3D1_set(dictionary *ini);
funPtr puAcc3D1KE_set(dictionary *ini);
funPtr puAccND1_set(dictionary *ini);
funPtr puAccND1KE_set(dictionary *ini);
void puAcc3D1(Population *pop, Grid *E);
void puAcc3D1KE(Population *pop, Grid *E);
void puAccND1(Population *pop, Grid *E);
void puAccND1KE(Population *pop, Grid *E);
/* Boris with a uniform external B (puBoris3D1/KE, pusher.c:394-483), the
 * reference's indexing defect corrected; puGet3DRotationParameters
 * (pusher.c:485-505) reads fields:BExt, population:charge/mass */
funPtr puBoris3D1_set(dictionary *ini);
funPtr puBoris3D1KE_set(dictionary *ini);
void puBoris3D1(Population *pop, Grid *E, const double *T, const double *S);
void puBoris3D1KE(Population *pop, Grid *E, const double *T, const double *S);
void puGet3DRotationParameters(dictionary *ini, double *T, double *S);
/* order 0, nearest grid point (pusher.c:310-391, 640-668, puInterpND0
 * :1164-1180); puAccND0_set returns puAccND0KE as in the reference */
funPtr puAccND0_set(dictionary *ini);
funPtr puAccND0KE_set(dictionary *ini);
funPtr puDistrND0_set(dictionary *ini);
void puAccND0KE(Population *pop, Grid *E);
void puDistrND0(const Population *pop, Grid *rho);
funPtr puDistr3D1_set(dictionary *ini);
funPtr puDistrND1_set(dictionary *ini);
void puDistr3D1(const Population *pop, Grid *rho);
void puDistrND1(const Population *pop, Grid *rho);
funPtr puExtractEmigrants3D_set(dictionary *ini);
funPtr puExtractEmigrantsND_set(dictionary *ini);
void puExtractEmigrants3D(Population *pop, MpiInfo *mpiInfo);
void puExtractEmigrantsND(Population *pop, MpiInfo *mpiInfo);
void puMigrate(Population *pop, MpiInfo *mpiInfo, Grid *grid);
int puNeighborToReciprocal(int neighbor, int nDims);
int puNeighborToRank(MpiInfo *mpiInfo, int neighbor);
int puRankToNeighbor(MpiInfo *mpiInfo, int rank);

/* --------------------------------------------------------- multigrid -- */
typedef struct MultigridSolver MultigridSolver;
void mgSolver(void (**solve)(), void *(**solverAlloc)(), void (**solverFree)());
funPtr mgSolver_set(dictionary *ini);
MultigridSolver *mgAllocSolver(const dictionary *ini, Grid *rho, Grid *phi);
void mgFreeSolver(MultigridSolver *solver);
void mgSolve(MultigridSolver *solver, Grid *rho, Grid *phi, const MpiInfo *mpiInfo);
long mgCycleCount(const MultigridSolver *solver);
/* diagnostics (not in the reference): cap the V-cycles of one solve
 * (0 = until converged, as multigrid.c:1698) and record the RMS residual
 * after each cycle of the last solve into a buffer of histCap entries;
 * mgHistory copies it out and returns the cycle count of that solve */
void mgSetLimit(MultigridSolver *solver, long maxCycles, long histCap);
long mgHistory(const MultigridSolver *solver, double *out, long cap);
int mgLevels(const MultigridSolver *solver);
/* halo planes of the sharded level 0 (multigrid:shard), 0 for a replicated solve */
int mgShardHalo(const MultigridSolver *solver);
/* multigrid:extrapolate with objects (two solves per step, main.c:230-238):
 * the initial guess of the NEXT solve only -- FIRST: extrapolated from the
 * first solutions of the last two steps; SECOND: this step's first solution
 * plus the last step's correction response; WARM: the reference's warm
 * start (any solve not announced, e.g. the capacitance matrix's).  Runs
 * without objects extrapolate every solve (SERIES) and ignore this. */
#define PINC_MG_GUESS_WARM 0
#define PINC_MG_GUESS_SERIES 1
#define PINC_MG_GUESS_FIRST 2
#define PINC_MG_GUESS_SECOND 3
void mgGuessNext(MultigridSolver *solver, int role);

/* ---------------------------------------------------------- spectral -- */
/* spectral.c:14-115; N-D extension of the reference's 1-D solver on rocFFT */
typedef struct SpectralSolver SpectralSolver;
void sSolver(void (**solve)(), void *(**solverAlloc)(), void (**solverFree)());
funPtr sSolver_set(dictionary *ini);
SpectralSolver *sAlloc(const dictionary *ini, Grid *rho, Grid *phi);
void sFree(SpectralSolver *solver);
void sSolve(SpectralSolver *solver, Grid *rho, Grid *phi, const MpiInfo *mpiInfo);
long sSolveCount(const SpectralSolver *solver);
/* 1 if the solve is slab-distributed (several ranks, 3-D), 0 if gathered */
int sSolveDistributed(const SpectralSolver *solver);

/* ------------------------------------------------ immersed objects -- */
/* object.c on the device (pinc_obj.c).  As main.c:95,
 * 126-127: oAlloc, then oOpenH5(ini, obj, mpiInfo, units, denorm, "test")
 * names <files:output>_test.grid.h5 and oReadH5 reads its /Object [nz,ny,nx,1]
 * (values 1..K) and builds the tables (object.c:717-756); a missing file or
 * an all-zero mask is a run without objects.  Extension: objects:sphere =
 * cx,cy,cz,r or objects:file = <.h5> in the ini builds them in oAlloc. */
Object *oAlloc(const dictionary *ini);
void oOpenH5(const dictionary *ini, Object *obj, const MpiInfo *mpiInfo, const Units *units, double denorm,
             const char *fName);
void oReadH5(Object *obj, const MpiInfo *mpiInfo);
void oCloseH5(Object *obj);
void oFree(Object *obj);
void oComputeCapacitanceMatrix(Object *obj, const dictionary *ini, const MpiInfo *mpiInfo);
void oApplyCapacitanceMatrix(Grid *rho, const Grid *phi, const Object *obj, const MpiInfo *mpiInfo);
void oCollectObjectCharge(Population *pop, Grid *rhoObj, Object *obj, const MpiInfo *mpiInfo);

/* ------------------------------------------------------- h5 output -- */
/* The reference's output files (grid.c:1161-1270, population.c:497-698,
 * io.c:566-734), written by rank 0 with serial HDF5 loaded at run time
 * (PINC_HDF5_LIB or libhdf5.so); hid_t is passed as long long and MPI_Op as
 * PINC_OP_SUM / PINC_OP_MAX. */
#define PINC_OP_SUM 0
#define PINC_OP_MAX 1
void gOpenH5(const dictionary *ini, Grid *grid, const MpiInfo *mpiInfo, const Units *units, double denorm,
             const char *fName);
void gWriteH5(const Grid *grid, const MpiInfo *mpiInfo, double n);
void gCloseH5(Grid *grid);
void pOpenH5(const dictionary *ini, Population *pop, const Units *units, const char *fName);
void pWriteH5(Population *pop, const MpiInfo *mpiInfo, double posN, double velN);
void pCloseH5(Population *pop);
long long xyOpenH5(const dictionary *ini, const char *fName);
void xyCreateDataset(long long h5, const char *name);
void xyWrite(long long h5, const char *name, double x, double y, int op);
void xyCloseH5(long long h5);
void pCreateEnergyDatasets(long long xy, Population *pop);
void pWriteEnergy(long long xy, Population *pop, double x);
int pinc_h5_available(void);
long pinc_h5_read(const char *path, const char *name, int isAttr, double *out, long cap);
int pinc_h5_dims(const char *path, const char *name, long *dimsOut);
int pinc_h5_write(const char *path, const char *name, int rank, const long *dims, const double *data);

/* ---------------------------------------------------------- run mode -- */
/* regular (main.c:50-304): one process per GPU, the world taken from the
 * launcher (pinc_boot.c: PINC_RANK/PINC_WORLD_SIZE, torchrun, Open MPI,
 * MPICH/PMI or Slurm variables; RCCL over xGMI, or PINC_TRANSPORT=host) */
void regular(dictionary *ini);
funPtr regular_set(dictionary *ini);
/* the reference's diagnostic run modes (multigrid.c:1731-1900, spectral.c:
 * 117-150) are outside this build's hot path: their
 * selectors exist so main.c's select list links; selecting one ends the run
 * with msg(ERROR) */
funPtr mgMode_set(dictionary *ini);
funPtr mgModeErrorScaling_set(dictionary *ini);
funPtr sMode_set(dictionary *ini);
/* a process that sets its world through PincSimOpts (Python, bench.py)
 * declares it before any other call, so that no launcher variable is read */
void pinc_world_explicit(void);

/* ====================================================== PincSim API ===== */
/* One process per GPU.  A simulation owns the ini, units, population, grids
 * and solver of one rank and runs main.c's loop (objects compiled out). */
typedef struct PincSim PincSim;

typedef struct {
	int literal;        /* 1: main.c's double FROMHALO add + extra solve */
	int perturb;        /* apply pPosPerturb at init (Langmuir runs) */
	int maxwell;        /* Maxwellian velocities from the counter RNG */
	int deviceInit;     /* generate the initial state on the device */
	unsigned long long seed;
	int rank, nranks;   /* slab decomposition along the last dimension */
	int device;         /* HIP device ordinal */
	const unsigned char *commId; /* PINC_COMM_ID_BYTES, NULL if nranks==1 */
	int timing;         /* record per-phase HIP events */
} PincSimOpts;

const char *pinc_last_error(void);
PincSim *pinc_sim_create(const char *iniPath, int nOver, const char **over, const PincSimOpts *opts);
void pinc_sim_free(PincSim *sim);
int pinc_sim_init(PincSim *sim);            /* initial conditions + fields + half step */
int pinc_sim_step(PincSim *sim);            /* one iteration of main.c:197-274 */
int pinc_sim_steps(PincSim *sim, int n);    /* n iterations without returning to the caller */
int pinc_sim_op(PincSim *sim, const char *op);
int pinc_sim_energy(PincSim *sim, double *ke, double *pe, double *keSpecies); /* rank-summed */
long pinc_sim_cycles(const PincSim *sim);
/* mgSetLimit / mgHistory of the simulation's multigrid solver (-1 if the
 * Poisson solver is spectral) */
int pinc_sim_mg_limit(PincSim *sim, long maxCycles, long histCap);
int pinc_sim_mg_levels(PincSim *sim);  /* levels of the multigrid hierarchy in use */
int pinc_sim_mg_shard(PincSim *sim);   /* mgShardHalo of the solver (0: replicated or spectral) */
int pinc_sim_spectral_distributed(PincSim *sim); /* sSolveDistributed (0 for multigrid) */
/* charge the immersed objects have collected since init (object.c:497
 * chargeCounter, summed over objects and ranks; 0 without objects) */
double pinc_sim_obj_collected(PincSim *sim);
long pinc_sim_mg_history(PincSim *sim, double *out, long cap);
int pinc_sim_nspecies(const PincSim *sim);
int pinc_sim_ndims(const PincSim *sim);
long pinc_sim_pop_count(PincSim *sim, int s);
int pinc_sim_pop_get(PincSim *sim, int s, double *pos, double *vel);
int pinc_sim_pop_set(PincSim *sim, int s, long n, const double *pos, const double *vel);
long pinc_sim_grid_shape(PincSim *sim, int which, int *size4);   /* 0 rho,1 phi,2 E */
int pinc_sim_grid_get(PincSim *sim, int which, double *out);
int pinc_sim_grid_set(PincSim *sim, int which, const double *in);
int pinc_sim_emigrants(PincSim *sim, long *nEmigrants);
int pinc_sim_species(PincSim *sim, double *charge, double *mass);
int pinc_sim_sync(PincSim *sim);
/* main.c's output (main.c:120-131, 262-266): open pop, rho, phi, E and the
 * history under files:output, then write them for step n (positions at n,
 * velocities at n+0.5, energies) -- what regular() does when files:h5 = 1 */
int pinc_sim_open_output(PincSim *sim);
int pinc_sim_write_output(PincSim *sim, double n);
/* per-phase device times accumulated since the last reset (ms):
 * 0 move+classify, 1 extract, 2 migrate, 3 deposit(+fold), 4 solve,
 * 5 efield, 6 accelerate, 7 energy */
#define PINC_NPHASES 8
int pinc_sim_timers(PincSim *sim, double *ms);
int pinc_sim_timers_reset(PincSim *sim);
/* Kernel probes: record HIP events around up to maxSamples launches of each
 * probed kernel on the library's stream, without host synchronisation; read
 * the mean duration and mean algorithmic bytes per launch afterwards.
 * Algorithmic bytes follow SURVEY.md 8(d).
 * pinc_probe_start(PINC_PROBE_ALL, n) probes every kernel below. */
#define PINC_PROBE_GS 0        /* red-black smoothing pass, finest level */
#define PINC_PROBE_ACCEL 1     /* gather + accelerate */
#define PINC_PROBE_MOVE 2      /* move + classify */
#define PINC_PROBE_DEPOSIT 3   /* charge deposit */
#define PINC_PROBE_RESIDUAL 4  /* residual norm, finest level */
#define PINC_PROBE_SPECTRAL 5  /* spectral solve (r2c + scale + c2r) */
#define PINC_PROBE_PUSH 6      /* fused kick + drift + classify + deposit */
#define PINC_PROBE_CYCLE 7     /* one V-cycle replayed as a graph (multigrid:graph) */
/* the launches of PINC_PROBE_PUSH by kind (each also counts in PUSH) */
#define PINC_PROBE_PUSH_PLAIN 8 /* fused push, output in input order */
#define PINC_PROBE_PUSH_COUNT 9 /* ... that also counts its output cells (before a sort) */
#define PINC_PROBE_PUSH_SORT 10 /* ... that writes its output in tile order */
#define PINC_NPROBES 11
#define PINC_PROBE_ALL (-1)
int pinc_probe_start(int kernel, int maxSamples);
int pinc_probe_read(int kernel, double *meanMs, double *meanBytes, int *samples, long *launches);
/* Duration (ms) of recorded launch i of a probed kernel, in launch order, and
 * its tag (PINC_PROBE_PUSH: species | kind << 8, kind 0 plain, 1 count,
 * 2 sort; 0 for the other kernels).  Returns 1 if i is not recorded. */
int pinc_probe_sample(int kernel, int i, double *ms, int *tag);
long pinc_sim_total_particles(PincSim *sim);

/* Host transport for the multi-rank collectives (testing and CI: several
 * processes on one GPU, where RCCL refuses duplicate devices).  When set
 * before pinc_sim_create, no RCCL communicator is made and every exchange,
 * allgather and allreduce stages device data through host memory and calls
 * these callbacks (0 = success).  exchange: op i sends sendBytes[i] to
 * sendPeer[i] and receives recvBytes[i] from recvPeer[i]; the peer's send
 * op i pairs with this rank's receive op i.  NULL restores RCCL. */
/* Statistics of the collectives by kind (0 halo: gHaloOp's plane exchanges,
 * 1 ext_halo: the sharded multigrid's deep halo, 2 migrate: migrant counts
 * and records, 3 allgather, 4 allreduce, 5 spectral_transpose: the slab
 * solve's all-to-all): start (up to maxCalls calls timed with HIP events on
 * the library's stream), then read device ms, this rank's payload bytes,
 * calls and timed calls per kind.  Returns PINC_COMM_KINDS, -1 if never
 * started. */
#define PINC_COMM_KINDS 6
int pinc_comm_stats_start(int maxCalls);
int pinc_comm_stats_read(double *ms, double *bytes, long *calls, long *timedCalls);
const char *pinc_comm_kind_name(int kind);

typedef struct {
	int (*exchange)(void *user, int nOps, const int *sendPeer, const void *const *sendbuf, const long *sendBytes,
	                const int *recvPeer, void *const *recvbuf, const long *recvBytes);
	int (*allgather)(void *user, const double *send, double *recv, long count);
	int (*allreduce_sum)(void *user, double *buf, long count);
	void *user;
} pinc_host_transport_t;
int pinc_set_host_transport(const pinc_host_transport_t *t);

#ifdef __cplusplus
}
#endif
#endif
