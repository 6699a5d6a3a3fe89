/*
 * pinc_internal.h -- private state behind include/pinc.h (host side, C).
 */
#ifndef PINC_INTERNAL_H
#define PINC_INTERNAL_H

/* system headers first: pinc.h defines the reference's select() macro */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/select.h>
#include "pinc.h"

#define PINC_NNE 27
#define PINC_PHASE_RING 64

typedef struct PincObj PincObj;

/* one process drives one GPU: stream, communicator and scratch are global,
 * as the reference relies on MPI_COMM_WORLD */
typedef struct {
	int initialised;
	int device;
	void *stream;
	void *comm;
	int rank, nranks;
	double *dScratch;   /* device: 8192 partials + 256 scalar slots */
	double *hPinned;    /* host, pinned: 32 doubles for the step's small reads */
	int *dErr;          /* device error word (asserts) */
	double maxVel;
	double thr[9];      /* migration thresholds lo[nd], up[nd], assert bound[nd] */
	int thrSet;
	int capturing; /* a stream capture is open: no event probes */
	int traceSort; /* PINC_TRACE_SORT: print the adaptive sort schedule */
	/* launches that can set the assert word (dErr), and that count when the
	 * word was last read: an unchanged word is not read again */
	unsigned long errSerial, errRead;
	int extractSkip; /* PINC_EXTRACT_SKIP=0 turns off skipping extractions the push counted empty */
	int flagsSparse; /* PINC_FLAGS_SPARSE=0: every push writes every particle's flag (pinc_pusher.c) */
	int verbose;        /* PINC_VERBOSE=n: progress every n V-cycles */
	int timing;
	/* phase timers: event pairs per phase, read when the ring is full or
	 * the totals are asked for (pinc_phase_flush), not at each phase end */
	void *ev[PINC_NPHASES][2 * PINC_PHASE_RING];
	int phaseN[PINC_NPHASES];
	double phaseMs[PINC_NPHASES];
	int phaseOpen[PINC_NPHASES];
	/* kernel probe: HIP events around launches of one kernel, read lazily
	 * (no host synchronisation inside the timed region) */
	int probeOn[PINC_NPROBES];      /* kernel probed? */
	int probeMax, probeN[PINC_NPROBES];  /* capacity, recorded pairs */
	void **probeEv[PINC_NPROBES];   /* 2*probeMax events per kernel */
	double *probeBytes[PINC_NPROBES]; /* algorithmic bytes of each recorded launch */
	long probeLaunches[PINC_NPROBES]; /* launches seen (recorded or not) */
	int *probeTag[PINC_NPROBES];     /* tag of each recorded launch (pinc_probe_tag) */
} PincCtx;

/* probe hooks around a launch of kernel k with algorithmic byte count b */
int pinc_probe_begin(int k);
void pinc_probe_count(int k);
void pinc_phase_flush(void);
void pinc_probe_end(int k, int slot, double bytes);
void pinc_probe_tag(int k, int slot, int tag);

extern PincCtx g_pinc;

#define PINC_PARTIALS 8192
#define PINC_SLOT(i) (g_pinc.dScratch + PINC_PARTIALS + (i))

struct PincDevPop {
	pinc_pop_t p;                 /* device pointers; ranges mirrored per call */
	long cap;                     /* total capacity */
	unsigned char *flags;
	int *chunkCount;              /* per species at chunkBase[s] */
	long chunkBase[PINC_MAX_SPECIES + 1];
	int flagsValid;
	/* what the flag bytes of species s's whole range hold (pinc_pusher.c,
	 * flags_before_write): PINC_FLAGS_CLEAN all the centre, so a push may
	 * write only its leavers' flags; PINC_FLAGS_PENDING the centre except at
	 * the particles the last write flagged, all below flagN[s]; else unknown */
	int flagState[PINC_MAX_SPECIES];
	long flagN[PINC_MAX_SPECIES];
	pinc_extract_ws_t ws[PINC_MAX_SPECIES];
	long nEmig[PINC_MAX_SPECIES];
	long neCount[PINC_MAX_SPECIES][PINC_NE_CODES]; /* directions + the object sink */
	double *qm, *mq;              /* device q/m and m/q per species */
	double *kePartial;
	pinc_geom_t geom;
	/* tiled layout (population:layout = tiled): particles sorted by tile
	 * every sortInterval moves into the alternate arrays, then swapped */
	int tiled, sortInterval, tileWidth;
	long moves;
	double *altX[3], *altV[3];
	int *sortWork[PINC_MAX_SPECIES];    /* per species: counts | cell ends | scan scratch */
	long sortWorkCap[PINC_MAX_SPECIES];
	long sortKeys;                      /* cells (keys) of the sort */
	long cellValid[PINC_MAX_SPECIES];   /* particles still in sorted order (-1: no sort yet) */
	/* fused push (population:fused, default 1): puAcc
	 * runs kick + drift + classify + deposit in one pass and leaves the moved
	 * positions in altX until the next puMove swaps them in; the charge of
	 * the particles that stayed is kept per species in rhoS until puDistr
	 * adds the immigrants and combines */
	int fused;
	int pending;                        /* altX holds the positions after the next move */
	int depValid;                       /* rhoS holds the last move's deposits */
	int depExtracted;                   /* ... and extract ran since (depEnd valid) */
	long depEnd[PINC_MAX_SPECIES];      /* particles [iStart, depEnd) are in rhoS */
	double *rhoS[PINC_MAX_SPECIES];
	long rhoN;
	/* tiled + fused: every push writes its output sorted by the cells of its
	 * input (counting sort folded into the push; the push also counts the
	 * cells of its output for the next one) */
	int sorted;
	int pendingSorted;                  /* pending velocities are in altV, in slot order */
	long nKeys;
	int *keyCnt[PINC_MAX_SPECIES];      /* cell counts of the current positions */
	int *keyNext[PINC_MAX_SPECIES];     /* counts being built by the push */
	int *keyCur[PINC_MAX_SPECIES];      /* cursors (exclusive offsets) */
	int *keyWork[PINC_MAX_SPECIES];     /* scan scratch */
	int cntValid[PINC_MAX_SPECIES];
	int everSorted;                     /* input already in cell order once */
	int permId[PINC_MAX_SPECIES];       /* species s left in order by the pending sorting push */
	/* particles each species' last push flagged to leave (emigrants,
	 * collected, outside the frame), read with the sort counters; emigValid:
	 * the current flags are that push's, so a species with none skips the
	 * extraction (no kernels, no host read; one rank, where the tiled push
	 * wraps every dimension in place) */
	unsigned long long *emigCnt;
	unsigned long long emigLast[PINC_MAX_SPECIES];
	int emigValid;
	/* the counter block (moved, spread, KE sums, emigrants) comes back
	 * asynchronously into pinned memory (hostCnt, cntEvent) and is taken in
	 * by pinc_pop_settle: at the next push, extraction, KE sum or energy
	 * read, whose own host wait usually covers it (no read of its own) */
	unsigned long long *hostCnt;
	void *cntEvent;
	int cntPending, cntE, keDeferred;
	int cntSortS[PINC_MAX_SPECIES], cntCountS[PINC_MAX_SPECIES];
	int vKicked[PINC_MAX_SPECIES];      /* p.v of species s holds the pending push's kicked velocities
	                                       (materialised before its E was written, pinc_grid_touch) */
	Grid *pendingE;                     /* E of the pending push's kick (pinc_pending_vel) */
	unsigned long long pendingESerial, pendingEGen; /* ... its serial and write count then */
	/* adaptive sort schedule (population:sortFraction > 0): a species is
	 * sorted once the fraction of its particles that left their cell since
	 * its last sort would pass sortFraction, at most sortMax pushes apart */
	double sortFraction;
	int sortMax;
	unsigned long long *movedCnt;       /* device, per species, this push */
	/* population:sortSpread > 0: a sort due by the displaced fraction waits
	 * until the blocks' mean input cell box has grown to sortSpread times its
	 * size in the first push after the last sort (a drifting beam changes
	 * cell without spreading); sortMax still bounds the interval */
	double sortSpread;
	unsigned long long *spreadCnt;      /* device, per species, this push (after movedCnt, then the
	                                     * kinetic-energy sums as doubles: one block, one read) */
	double keSums[PINC_MAX_SPECIES];    /* host: this push's v^2 sums, read with the counters */
	int keSumsValid;
	double spreadBase[PINC_MAX_SPECIES], spreadLast[PINC_MAX_SPECIES];
	double movedFrac[PINC_MAX_SPECIES], lastRate[PINC_MAX_SPECIES];
	int sinceSort[PINC_MAX_SPECIES], sortNext[PINC_MAX_SPECIES];
	/* fused object collection (pinc_obj_attach): the push flags a particle
	 * that enters an object PINC_NE_SINK (removed by the next extract, not
	 * deposited) and counts it in objCount[s * objK + id - 1] */
	const unsigned char *objInside;
	long objSy, objSz, objNodes;
	int *objCount;
	int objK;
	PincObj *objOwner;                  /* the object set attached (pFree detaches it) */
	int objLo[3], objHi[3];
	/* the host mirror was written (pPosLattice, pPosPerturb, pVelZero,
	 * pVelMaxwell) and is the truth until the next device operator uploads
	 * it (pinc_pop_flush_host): main.c never calls pSyncToDevice */
	int hostDirty;
	/* multi-rank migration buffers (AoS records: nd pos, nd vel, ne) */
	double *sendBuf[2], *recvBuf[2];
	long sendCap, recvCap;
};

struct PincDevGrid {
	int nValues;
	double *d;          /* slab storage [nloc+2] planes (nValues per node) */
	long n;             /* elements of d */
	long planeSize;     /* nodes per plane */
	pinc_geom_t geom;
	double *global;     /* global periodic view (rho, phi) */
	int ownsGlobal;
	int globalIsTruth;  /* the solver writes global (phi): the slab follows by TOHALO; for rho
	                       the slab is the truth and global its gathered copy */
	int ghostsValid;    /* slab ghost planes already hold periodic images */
	double *recv[2];    /* halo receive planes (multi-rank) */
	double *scaled;     /* E as rescaled for the species being pushed (lazy) */
	double *scaledAll;  /* every species' rescaled E, one pass per push round (lazy) */
	int scaledAllS;     /* species it holds room for */
	/* sharded multigrid (phi only): this rank's slab with extOff halo planes
	 * on each side, extPlanes planes in all, owned by the solver */
	double *ext;
	int extOff, extPlanes;
	int extStale;       /* owned planes written (gSyncToDevice), halo not yet refreshed */
	/* main.c's second gHaloOp(addSlice, rho, FROMHALO) of a step
	 * (main.c:226,232): the population of the last deposit, its order (0 NGP,
	 * 1 CIC) and the folds since; lit is the scratch of the missing weight */
	const Population *depPop;
	int depOrder, folds;
	double *lit;
	/* writes of d since gAlloc, and a process-unique id with the list of live
	 * grids: a pending sorting push checks that its E is the one it kicked
	 * with (pinc_pending_vel) */
	unsigned long long gen, serial;
	PincDevGrid *liveNext;
};
enum { PINC_FLAGS_UNKNOWN = 0, PINC_FLAGS_CLEAN = 1, PINC_FLAGS_PENDING = 2 };
int pinc_flags_before_write(Population *pop, int s, int sparseOk);
void pinc_flags_after_extract(Population *pop, int s, long nBefore);
/* d is about to be rewritten: a pending sorting push that kicked with this
 * grid first materialises its kicked velocities (pinc_pusher.c).  EVERY
 * operator that writes a grid's device data must call this first (gMul,
 * gFinDiff1st, gHaloOp, gSyncToDevice, gFree do): gen only moves here, so
 * the re-kick's guard cannot see a write that skips it. */
void pinc_grid_touch(Grid *g);
/* populations whose pending sorting push may need its E (pinc_pusher.c) */
void pinc_pending_register(Population *pop);
/* take in the last push's counter block (waits for its copy if needed) */
void pinc_pop_settle(Population *pop);
void pinc_pending_unregister(Population *pop);
/* the grid is allocated and is the one with this serial */
int pinc_grid_live(const Grid *g, unsigned long long serial);

/* immersed objects (pinc_obj.c; object.c, config C5) */
PincObj *pinc_obj_create(const dictionary *ini, const Grid *rho);
void pinc_obj_free(PincObj *o);
void pinc_obj_capacitance(PincObj *o, Grid *rho, Grid *phi, void *solver,
                          void (*solve)(void *, Grid *, Grid *, const MpiInfo *), const MpiInfo *mpi);
void pinc_obj_collect(PincObj *o, Population *pop, int discard);
void pinc_obj_add_rho(PincObj *o, Grid *rho);
void pinc_obj_attach(PincObj *o, Population *pop);
double pinc_obj_apply(PincObj *o, Grid *rho, const Grid *phi);
long pinc_obj_nsurface(const PincObj *o);
/* the attached population is being freed (main.c frees pop before obj) */
void pinc_obj_forget_pop(PincObj *o);
/* slab-distributed Poisson solve with a slab plan (pinc_spectral.c) */
void pinc_slab_poisson(pinc_fft_slab_t *plan, const double *rhoSlab, double *phiSlab, const char *what);
double pinc_obj_collected(const PincObj *o);
/* Boris selected through methods:acc: its initial half step (pinc_regular.c) */
void pinc_boris_half_step(int on);
int pinc_boris_selected(funPtr acc);

struct MultigridSolver {
	int nLevels, nPre, nPost, nCoarse, mgCycles;
	int pre3d, post3d, coarse3d, restr3d;
	pinc_lvl_t L[PINC_MAX_LEVELS];
	long N[PINC_MAX_LEVELS];
	double *rho[PINC_MAX_LEVELS], *phi[PINC_MAX_LEVELS], *res[PINC_MAX_LEVELS];
	/* native smoothing ping-pongs phi[q] and res[q] by swapping the
	 * pointers; swapped[q] = 1 while they are exchanged (pp_restore) */
	int swapped[PINC_MAX_LEVELS];
	long cycles;
	Grid *rhoGrid, *phiGrid;
	int native;
	int useGraph;      /* multigrid:graph: replay one captured V-cycle */
	void *cycleGraph;  /* instantiated graph of vrec(S, 0) */
	/* diagnostics: RMS residual after each V-cycle of the last solve, and an
	 * optional cap on the cycles of one solve (0 = loop until converged) */
	double *hist;
	long histCap, histN, maxCycles;
	long fusedMin;     /* smallest level (points) smoothed by the fused sweeps */
	/* multigrid:extrapolate: level-0 initial guesses (pinc_mg.c guess_*).
	 * Runs without objects: 2 phi_n - phi_{n-1} (phiPrev holds phi_{n-1};
	 * havePrev counts the solves seen, up to 2).  Runs with objects (two
	 * solves per step, mgGuessNext): the first from the first solves of the
	 * last two steps (phiA, phiB), the second as the first plus the last
	 * step's correction response (dCorr = its second minus its first
	 * solution); any other solve keeps the warm start. */
	int extrap, havePrev, objects, role, haveCorr;
	double *phiPrev, *phiA, *phiB, *dCorr;
	/* objects:secondGuess = spectral (one rank): the second solve of a step
	 * starts from the first solution plus the exact discrete response to
	 * the correction charge (rocFFT, the 7-point symbol); rhoSave holds the
	 * first solve's rho */
	int secondSpectral;
	double *rhoSave, *dphi;
	pinc_fft_t *fft;
	pinc_fft_slab_t *fftSlab; /* secondSpectral == 2: the sharded level 0's transform */
	/* multigrid:spectralCoarse (native mode): level 1's correction solved
	 * exactly (rocFFT, the 7-point symbol) instead of by the levels below */
	pinc_fft_t *fftCoarse;
	/* sharded level 0 (native mode, multigrid:shard):
	 * rho[0]/phi[0]/res[0] are this rank's z-slab with hz halo planes on
	 * each side (L[0], N[0] = that extended slab), levels >= 1 global */
	int shard, hz, chunk, nloc0;
	long ps0, Ng0;                 /* plane size, global level-0 points */
	int z0;                        /* global plane of extended plane 0 */
	double *rho1Slab;              /* this rank's level-1 planes before the all-gather */
	pinc_lvl_t L1s;
	/* sharded level 0 with multigrid:spectralCoarse: level 1 stays
	 * decomposed (dist1), as the reference keeps every level on its
	 * subdomain (mgAllocSubGrids, multigrid.c:128): the correction of this
	 * rank's level-1 planes comes from the slab-distributed transform
	 * (fftCoarseSlab; all-to-all transposes instead of an all-gather of
	 * level 1) into phi1Ext, which holds one halo plane on each side for the
	 * prolongation of the owned level-0 planes */
	int dist1;
	pinc_fft_slab_t *fftCoarseSlab;
	double *phi1Ext;
	/* the per-cycle norm read without idling the GPU (mgSolve): the norm
	 * goes to pinned memory asynchronously and, while the host waits for
	 * it, the next cycle's first double sweep (phi -> res, which leaves phi
	 * untouched) is already queued; preDone tells that cycle's pre-smoothing
	 * the sweep is done.  Only when the last solve of this role needed more
	 * cycles than have run (lastCycles), so a converged solve rarely leaves a
	 * sweep unused.  (multigrid:speculate, default 1; native, replicated, no
	 * graph.) */
	int speculate, preDone;
	long lastCycles[4];
	double *hostNorm;
	void *normEvent;
	/* a small 2-D solve on one rank runs its V-cycles and the convergence
	 * test in one workgroup (pinc_hip_mg_solve_small): the cycle count, the
	 * last residual and the history come back in one read (smallOut, pinned
	 * hostSmall) per launch */
	int small;
	double *smallOut, *hostSmall;
	double *smallBasis; /* with multigrid:spectralCoarse: level 1's Fourier basis and eigenvalues */
};

/* gFinDiff1st and gMul(field, -1) in one pass, bit for bit the two
 * (pinc_grid.c; regular()'s step) */
void pinc_fin_diff_neg(const Grid *scalar, Grid *field);

/* collectives over RCCL or the host transport (pinc_comm.c) */
void pinc_comm_exchange(int nOps, const int *sendPeer, void *const *sendbuf, const long *sendBytes,
                        const int *recvPeer, void *const *recvbuf, const long *recvBytes, const char *what);
void pinc_comm_allgather(const double *send, double *recv, long count, const char *what);
void pinc_comm_allreduce_sum(double *buf, long count, const char *what);
int pinc_comm_host_transport(void);
void pinc_ext_halo(double *a, long ps, int nloc, int h);

/* process world and device context (pinc_boot.c, pinc_core.c) */
int pinc_boot_world(void);
void pinc_boot_configured(void);
const char *pinc_launcher_env(int *rank, int *size, int *local);
void pinc_ctx_init(void);

/* upload a host-written population before a device operator reads it */
void pinc_pop_flush_host(const Population *pop);
/* the weight a deposit without the literal factor misses for the second fold
 * of main.c:232 (pinc_pusher.c) */
/* kicked velocities pending after a sorting push, in the current order */
void pinc_pot_energy_launch(const Grid *rho, const Grid *phi);
void pinc_pending_vel(const Population *pop, int s, double *const *dst);
void pinc_literal_second_fold(const Population *pop, Grid *rho, int order);

/* helpers shared by the host translation units */
void pinc_ctx_require(void);
void pinc_check(int rc, const char *where);
void pinc_phase_begin(int phase);
void pinc_phase_end(int phase);
pinc_geom_t pinc_geom_from_grid(const Grid *g, const MpiInfo *mpi);
pinc_geom_t pinc_geom_current(void);
void pinc_geom_set(pinc_geom_t g);
pinc_pop_t pinc_devpop(const Population *pop);
double pinc_reduce_host(int nParts, double div);
int pinc_ipow3(int d);

#endif
