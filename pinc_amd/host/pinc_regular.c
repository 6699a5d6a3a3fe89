/*
 * pinc_regular.c -- the PIC run mode (main.c:50-304 with the immersed-object
 * hooks compiled out) on the MI355X operator surface, and
 * the PincSim C API that Python (bench.py, tests) drives through ctypes.
 *
 * Loop order per step (main.c:197-274, single-add harness of SURVEY.md
 * Appendix A; literal=1 adds main.c:231-235's second FROMHALO add and the
 * extra solve):
 *   puMove -> extractEmigrants -> puMigrate -> distr -> gHaloOp(add,rho,FROM)
 *   -> solve -> gHaloOp(set,phi,TO) -> gFinDiff1st -> gHaloOp(set,E,TO)
 *   -> gMul(E,-1) -> acc (+KE) -> pSumKinEnergy -> gPotEnergy
 * The per-step asserts pVelAssertMax / pPosAssertInLocalFrame are folded into
 * the move kernel and checked once per step.
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>

funPtr regular_set(dictionary *ini) {
	(void)ini;
	return (funPtr)regular;
}

/* main.c:32-35 also offers the reference's diagnostic run modes (multigrid
 * convergence studies, multigrid.c:1731-1900; the spectral check,
 * spectral.c:117-150).  They are outside the hot path;
 * the selectors exist so that main.c links against this library unchanged */
static void mode_unavailable(const char *name) {
	msg(ERROR, "methods:mode=%s is a diagnostic run mode of the reference that this build does not provide "
	           "(use methods:mode=regular)", name);
}
static void mgMode(dictionary *ini) { (void)ini; mode_unavailable("mgMode"); }
static void mgModeErrorScaling(dictionary *ini) { (void)ini; mode_unavailable("mgModeErrorScaling"); }
static void sMode(dictionary *ini) { (void)ini; mode_unavailable("sMode"); }
funPtr mgMode_set(dictionary *ini) { (void)ini; return (funPtr)mgMode; }
funPtr mgModeErrorScaling_set(dictionary *ini) { (void)ini; return (funPtr)mgModeErrorScaling; }
funPtr sMode_set(dictionary *ini) { (void)ini; return (funPtr)sMode; }

struct PincSim {
	dictionary *ini;
	Units *units;
	MpiInfo *mpi;
	Population *pop;
	Grid *E, *rho, *phi;
	void *solver;
	void (*solve)(void *, Grid *, Grid *, const MpiInfo *);
	void (*solverFree)(void *);
	int spectral;
	void (*acc)(Population *, Grid *);
	void (*distr)(const Population *, Grid *);
	void (*extractEmigrants)(Population *, MpiInfo *);
	PincSimOpts opts;
	int initialised;
	long steps;
	PincObj *obj;      /* immersed object (objects:sphere), or NULL */
	int output;        /* pinc_sim_open_output ran: files below are open */
	long long history;
};

static int g_simActive = 0;

static void report_errors(int err) {
	if (err & 1) msg(ERROR, "Particle travels too fast (population:maxVel exceeded, population.c:342-365)");
	if (err & 2) msg(ERROR, "Particle is out of bounds after migration (population.c:316-340)");
}

/* pPosAssertInLocalFrame's read of the assert word, unless no launch that
 * can set it ran since the word was last read (the step's closing read
 * covers the push that made this step's move) */
static void check_errors(void) {
	if (g_pinc.errSerial == g_pinc.errRead) return;
	int err = 0;
	g_pinc.errRead = g_pinc.errSerial;
	pinc_check(pinc_hip_d2h(&err, g_pinc.dErr, sizeof(int), g_pinc.stream), "assert word");
	report_errors(err);
}

static PincSim *sim_build(dictionary *ini, const PincSimOpts *opts) {
	PincSim *S = calloc(1, sizeof(*S));
	S->ini = ini;
	if (opts) {
		/* the caller sets the world (PincSimOpts: rank, size, device, RCCL id) */
		S->opts = *opts;
		if (S->opts.nranks < 1) S->opts.nranks = 1;
		pinc_boot_configured();
		g_pinc.device = S->opts.device;
		g_pinc.rank = S->opts.rank;
		g_pinc.nranks = S->opts.nranks;
		g_pinc.timing = S->opts.timing;
		pinc_ctx_require();
		if (S->opts.nranks > 1 && !g_pinc.comm && !pinc_comm_host_transport()) {
			if (!S->opts.commId) msg(ERROR, "multi-rank run without a communicator id");
			pinc_check(pinc_hip_comm_init(&g_pinc.comm, S->opts.commId, S->opts.nranks, S->opts.rank), "comm init");
		}
	} else {
		/* regular() as main.c runs it: the world comes from the launcher
		 * (mpirun, torchrun, srun or PINC_RANK/PINC_WORLD_SIZE), DESIGN.md 7 */
		S->opts.perturb = 1;
		pinc_boot_world();
		S->opts.rank = g_pinc.rank;
		S->opts.nranks = g_pinc.nranks;
		S->opts.device = g_pinc.device;
	}
	/* method selection (main.c:55-79) */
	S->acc = (void (*)(Population *, Grid *))select(ini, "methods:acc", puAcc3D1_set, puAcc3D1KE_set, puAccND1_set,
	                                                 puAccND1KE_set, puBoris3D1_set, puBoris3D1KE_set);
	S->distr = (void (*)(const Population *, Grid *))select(ini, "methods:distr", puDistr3D1_set, puDistrND1_set);
	S->extractEmigrants = (void (*)(Population *, MpiInfo *))select(ini, "methods:migrate", puExtractEmigrants3D_set,
	                                                                puExtractEmigrantsND_set);
	void (*solverInterface)() = select(ini, "methods:poisson", mgSolver_set, sSolver_set);
	void (*solve)() = NULL;
	void *(*solverAlloc)() = NULL;
	void (*solverFree)() = NULL;
	((void (*)(void (**)(), void *(**)(), void (**)()))solverInterface)(&solve, &solverAlloc, &solverFree);
	/* normalisation and allocation (main.c:84-107) */
	S->units = uAlloc(ini);
	uNormalize(ini, S->units);
	S->mpi = gAllocMpi(ini);
	S->pop = pAlloc(ini);
	S->E = gAlloc(ini, VECTOR);
	S->rho = gAlloc(ini, SCALAR);
	S->phi = gAlloc(ini, SCALAR);
	S->solver = ((void *(*)(const dictionary *, Grid *, Grid *))solverAlloc)(ini, S->rho, S->phi);
	S->solve = (void (*)(void *, Grid *, Grid *, const MpiInfo *))solve;
	S->solverFree = (void (*)(void *))solverFree;
	S->spectral = solve == (void (*)())sSolve;
	S->obj = pinc_obj_create(ini, S->rho);
	if (S->obj) pinc_obj_attach(S->obj, S->pop);
	if (S->opts.literal) {
		/* main.c:226,232 fold rho's ghosts twice; see literal_ghost_weights */
		S->pop->dev->geom.literal = 1;
		S->rho->dev->geom.literal = 1;
	}
	gCreateNeighborhood(ini, S->mpi, S->rho);
	gSetBndSlices(S->phi, S->mpi);
	g_pinc.maxVel = iniHas(ini, "population:maxVel") ? iniGetDouble(ini, "population:maxVel") : INFINITY;
	return S;
}

static void sim_init(PincSim *S) {
	Population *pop = S->pop;
	if (S->opts.deviceInit) {
		pInitDevice(S->ini, pop, S->mpi, S->opts.perturb, S->opts.maxwell, S->opts.seed);
	} else {
		pPosLattice(S->ini, pop, S->mpi);
		if (S->opts.maxwell) pVelMaxwell(S->ini, pop, S->opts.seed);
		else pVelZero(pop);
		if (S->opts.perturb) pPosPerturb(S->ini, pop, S->mpi);
		pSyncToDevice(pop);
	}
	S->extractEmigrants(pop, S->mpi);
	puMigrate(pop, S->mpi, S->rho);
	if (S->obj) {
		/* capacitance matrix, then main.c:163-166: particles that start
		 * inside the object are removed, their charge dropped */
		pinc_phase_begin(4);
		pinc_obj_capacitance(S->obj, S->rho, S->phi, S->solver, S->solve, S->mpi);
		pinc_phase_end(4);
		pinc_obj_collect(S->obj, pop, 1);
	}
}

static void sim_fields(PincSim *S) {
	/* main.c:168-186: one FROMHALO here, also in the literal loop */
	int lit = S->rho->dev->geom.literal;
	S->rho->dev->geom.literal = 0;
	S->distr(S->pop, S->rho);
	S->rho->dev->geom.literal = lit;
	gHaloOp((funPtr)addSlice, S->rho, S->mpi, FROMHALO);
	S->solve(S->solver, S->rho, S->phi, S->mpi);
	pinc_phase_begin(5);
	gFinDiff1st(S->phi, S->E);
	gHaloOp((funPtr)setSlice, S->E, S->mpi, TOHALO);
	gMul(S->E, -1.);
	pinc_phase_end(5);
	gMul(S->E, 0.5);
	int bor = pinc_boris_selected((funPtr)S->acc);
	if (bor) pinc_boris_half_step(1);
	S->acc(S->pop, S->E);
	if (bor) pinc_boris_half_step(0);
	gMul(S->E, 2.0);
}

static void sim_step(PincSim *S) {
	Population *pop = S->pop;
	puMove(pop, NULL);
	S->extractEmigrants(pop, S->mpi);
	puMigrate(pop, S->mpi, S->rho);
	/* pPosAssertInLocalFrame (main.c:219) before anything deposits an
	 * immigrant: a particle outside the local frame must not reach the
	 * deposit's grid indexing */
	check_errors();
	if (S->obj) pinc_obj_collect(S->obj, pop, 0); /* main.c:222 */
	S->distr(pop, S->rho);
	gHaloOp((funPtr)addSlice, S->rho, S->mpi, FROMHALO);
	if (S->obj) {
		/* main.c:230-238: rho += rhoObj (folded again in the literal
		 * loop), solve, capacitance correction, solve */
		pinc_obj_add_rho(S->obj, S->rho);
		if (S->opts.literal) gHaloOp((funPtr)addSlice, S->rho, S->mpi, FROMHALO);
		if (!S->spectral) mgGuessNext(S->solver, PINC_MG_GUESS_FIRST);
		S->solve(S->solver, S->rho, S->phi, S->mpi);
		pinc_obj_apply(S->obj, S->rho, S->phi);
		if (!S->spectral) mgGuessNext(S->solver, PINC_MG_GUESS_SECOND);
	} else if (S->opts.literal) {
		gHaloOp((funPtr)addSlice, S->rho, S->mpi, FROMHALO);
		S->solve(S->solver, S->rho, S->phi, S->mpi);
	}
	S->solve(S->solver, S->rho, S->phi, S->mpi);
	pinc_phase_begin(5);
	gHaloOp((funPtr)setSlice, S->phi, S->mpi, TOHALO);
	/* gFinDiff1st, gHaloOp(E), gMul(E, -1): the negation in the finite
	 * difference's own pass (exact, so it commutes with the halo copy) */
	pinc_fin_diff_neg(S->phi, S->E);
	gHaloOp((funPtr)setSlice, S->E, S->mpi, TOHALO);
	pinc_phase_end(5);
	S->acc(pop, S->E);
	pinc_phase_begin(7);
	/* gPotEnergy and the error word in one read (PINC_SLOT(3..4)); the
	 * push's counters and kinetic energies, copied before it, are in by then
	 * (pSumKinEnergy takes them in without a wait of its own) */
	pinc_pot_energy_launch(S->rho, S->phi);
	pinc_check(pinc_hip_d2d(PINC_SLOT(4), g_pinc.dErr, sizeof(int), g_pinc.stream), "assert word");
	g_pinc.errRead = g_pinc.errSerial;
	/* (into pinned memory: no staging copy on the host's wake-up path) */
	double *r = g_pinc.hPinned;
	pinc_check(pinc_hip_d2h(r, PINC_SLOT(3), 2 * sizeof(double), g_pinc.stream), "potential energy");
	pSumKinEnergy(pop);
	pop->potEnergy[pop->nSpecies] = 0.5 * r[0];
	pinc_phase_end(7);
	int err = 0;
	memcpy(&err, &r[1], sizeof(err));
	report_errors(err);
	S->steps++;
}

static void output_close(PincSim *S) {
	if (!S->output) return;
	pCloseH5(S->pop);
	gCloseH5(S->rho);
	gCloseH5(S->phi);
	gCloseH5(S->E);
	xyCloseH5(S->history);
	S->output = 0;
}

/* main.c:118-131: pop, rho, phi, E and history files, denorm 1 */
static void output_open(PincSim *S) {
	if (S->output) return;
	double denorm = 1.;
	pOpenH5(S->ini, S->pop, S->units, "pop");
	gOpenH5(S->ini, S->rho, S->mpi, S->units, denorm, "rho");
	gOpenH5(S->ini, S->phi, S->mpi, S->units, denorm, "phi");
	gOpenH5(S->ini, S->E, S->mpi, S->units, denorm, "E");
	S->history = xyOpenH5(S->ini, "history");
	pCreateEnergyDatasets(S->history, S->pop);
	S->output = 1;
}

/* main.c:262-266 */
static void output_write(PincSim *S, double n) {
	gWriteH5(S->E, S->mpi, n);
	gWriteH5(S->rho, S->mpi, n);
	gWriteH5(S->phi, S->mpi, n);
	pWriteH5(S->pop, S->mpi, n, n + 0.5);
	pWriteEnergy(S->history, S->pop, n);
}

static void sim_free(PincSim *S) {
	if (!S) return;
	output_close(S);
	pinc_obj_free(S->obj);
	if (S->solverFree) S->solverFree(S->solver);
	gFree(S->E);
	gFree(S->rho);
	gFree(S->phi);
	pFree(S->pop);
	gFreeMpi(S->mpi);
	uFree(S->units);
	iniClose(S->ini);
	free(S);
}

/* main.c:50-304 as a run mode of this library */
void regular(dictionary *ini) {
	PincSim *S = sim_build(ini, NULL);
	sim_init(S);
	sim_fields(S);
	/* the reference writes rho, phi, E, the particles and the energies every
	 * step (main.c:262-266); here only with files:h5 = 1, since at C4 that
	 * is tens of GB per step */
	int h5 = iniHas(ini, "files:h5") && iniGetInt(ini, "files:h5");
	if (h5) output_open(S);
	int nTimeSteps = iniGetInt(ini, "time:nTimeSteps");
	for (int n = 1; n <= nTimeSteps; n++) {
		msg(STATUS, "Computing time-step %i", n);
		sim_step(S);
		/* summed over the ranks, as pWriteEnergy's MPI_SUM rows (population.c:658-698) */
		double ke, pe;
		pinc_sim_energy(S, &ke, &pe, NULL);
		msg(STATUS, "KE %.17g PE %.17g", ke, pe);
		if (h5) output_write(S, (double)n);
	}
	S->ini = NULL; /* owned by the caller */
	sim_free(S);
}

/* ======================================================= PincSim API ===== */
PincSim *pinc_sim_create(const char *iniPath, int nOver, const char **over, const PincSimOpts *opts) {
	if (g_simActive) {
		msg(WARNING, "one simulation per process (the device context is global)");
		return NULL;
	}
	char **argv = calloc(nOver + 2, sizeof(char *));
	argv[0] = "pinc";
	argv[1] = (char *)iniPath;
	for (int i = 0; i < nOver; i++) argv[2 + i] = (char *)over[i];
	dictionary *ini = iniOpen(nOver + 2, argv);
	free(argv);
	PincSim *S = sim_build(ini, opts);
	g_simActive = 1;
	return S;
}

void pinc_sim_free(PincSim *S) {
	sim_free(S);
	g_simActive = 0;
}

int pinc_sim_init(PincSim *S) {
	sim_init(S);
	sim_fields(S);
	S->initialised = 1;
	return 0;
}

int pinc_sim_step(PincSim *S) {
	sim_step(S);
	return 0;
}

int pinc_sim_steps(PincSim *S, int n) {
	for (int i = 0; i < n; i++) sim_step(S);
	return 0;
}

int pinc_sim_op(PincSim *S, const char *op) {
	if (!strcmp(op, "init_particles")) sim_init(S);
	else if (!strcmp(op, "init_fields")) sim_fields(S);
	else if (!strcmp(op, "move")) puMove(S->pop, NULL);
	else if (!strcmp(op, "extract")) S->extractEmigrants(S->pop, S->mpi);
	else if (!strcmp(op, "migrate")) puMigrate(S->pop, S->mpi, S->rho);
	else if (!strcmp(op, "distr_nohalo")) S->distr(S->pop, S->rho);
	else if (!strcmp(op, "distr")) {
		S->distr(S->pop, S->rho);
		gHaloOp((funPtr)addSlice, S->rho, S->mpi, FROMHALO);
	} else if (!strcmp(op, "solve")) S->solve(S->solver, S->rho, S->phi, S->mpi);
	else if (!strcmp(op, "efield")) {
		gHaloOp((funPtr)setSlice, S->phi, S->mpi, TOHALO);
		gFinDiff1st(S->phi, S->E);
		gHaloOp((funPtr)setSlice, S->E, S->mpi, TOHALO);
		gMul(S->E, -1.);
	} else if (!strcmp(op, "efield_fused")) {
		/* the step's form (sim_step) */
		gHaloOp((funPtr)setSlice, S->phi, S->mpi, TOHALO);
		pinc_fin_diff_neg(S->phi, S->E);
		gHaloOp((funPtr)setSlice, S->E, S->mpi, TOHALO);
	} else if (!strcmp(op, "acc")) S->acc(S->pop, S->E);
	else if (!strcmp(op, "energy")) {
		pSumKinEnergy(S->pop);
		gPotEnergy(S->rho, S->phi, S->pop);
	} else if (!strcmp(op, "step")) sim_step(S);
	else {
		msg(WARNING, "unknown op %s", op);
		return 1;
	}
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), op);
	return 0;
}

int pinc_sim_energy(PincSim *S, double *ke, double *pe, double *keSpecies) {
	pinc_pop_settle(S->pop);
	int ns = S->pop->nSpecies;
	double v[PINC_MAX_SPECIES + 2];
	v[0] = S->pop->kinEnergy[ns];
	v[1] = S->pop->potEnergy[ns];
	for (int s = 0; s < ns; s++) v[2 + s] = S->pop->kinEnergy[s];
	if (g_pinc.nranks > 1) {
		double *d = PINC_SLOT(96);
		pinc_check(pinc_hip_h2d(d, v, (ns + 2) * sizeof(double), g_pinc.stream), "energy");
		pinc_comm_allreduce_sum(d, ns + 2, "energy allreduce");
		pinc_check(pinc_hip_d2h(v, d, (ns + 2) * sizeof(double), g_pinc.stream), "energy");
	}
	*ke = v[0];
	*pe = v[1];
	if (keSpecies)
		for (int s = 0; s < ns; s++) keSpecies[s] = v[2 + s];
	return 0;
}

/* V-cycles run so far (multigrid) or solves (spectral) */
long pinc_sim_cycles(const PincSim *S) {
	return S->spectral ? sSolveCount(S->solver) : mgCycleCount(S->solver);
}
int pinc_sim_mg_limit(PincSim *S, long maxCycles, long histCap) {
	if (S->spectral) return -1;
	mgSetLimit(S->solver, maxCycles, histCap);
	return 0;
}

int pinc_sim_mg_levels(PincSim *S) { return S->spectral ? 0 : mgLevels(S->solver); }
int pinc_sim_mg_shard(PincSim *S) { return S->spectral ? 0 : mgShardHalo(S->solver); }
int pinc_sim_spectral_distributed(PincSim *S) { return S->spectral ? sSolveDistributed(S->solver) : 0; }
double pinc_sim_obj_collected(PincSim *S) { return pinc_obj_collected(S->obj); }

long pinc_sim_mg_history(PincSim *S, double *out, long cap) {
	if (S->spectral) return -1;
	return mgHistory(S->solver, out, cap);
}

int pinc_sim_nspecies(const PincSim *S) { return S->pop->nSpecies; }
int pinc_sim_ndims(const PincSim *S) { return S->pop->nDims; }
long pinc_sim_pop_count(PincSim *S, int s) { return S->pop->iStop[s] - S->pop->iStart[s]; }

long pinc_sim_total_particles(PincSim *S) {
	long n = 0;
	for (int s = 0; s < S->pop->nSpecies; s++) n += S->pop->iStop[s] - S->pop->iStart[s];
	return n;
}

int pinc_sim_pop_get(PincSim *S, int s, double *pos, double *vel) {
	Population *p = S->pop;
	pSyncToHost(p);
	long a = p->iStart[s], n = p->iStop[s] - a, nd = p->nDims;
	if (pos) memcpy(pos, p->pos + a * nd, n * nd * sizeof(double));
	if (vel) memcpy(vel, p->vel + a * nd, n * nd * sizeof(double));
	return 0;
}

int pinc_sim_pop_set(PincSim *S, int s, long n, const double *pos, const double *vel) {
	Population *p = S->pop;
	if (n > p->iStart[s + 1] - p->iStart[s]) {
		msg(WARNING, "pinc_sim_pop_set: capacity exceeded");
		return 1;
	}
	pSyncToHost(p);
	long a = p->iStart[s], nd = p->nDims;
	memcpy(p->pos + a * nd, pos, n * nd * sizeof(double));
	memcpy(p->vel + a * nd, vel, n * nd * sizeof(double));
	p->iStop[s] = a + n;
	pSyncToDevice(p);
	return 0;
}

static Grid *which_grid(PincSim *S, int which) {
	return which == 0 ? S->rho : (which == 1 ? S->phi : S->E);
}

long pinc_sim_grid_shape(PincSim *S, int which, int *size4) {
	Grid *g = which_grid(S, which);
	for (int d = 0; d < 4; d++) size4[d] = d < g->rank ? g->size[d] : 1;
	return g->sizeProd[g->rank];
}

int pinc_sim_grid_get(PincSim *S, int which, double *out) {
	Grid *g = which_grid(S, which);
	gSyncToHost(g);
	memcpy(out, g->val, g->sizeProd[g->rank] * sizeof(double));
	return 0;
}

int pinc_sim_grid_set(PincSim *S, int which, const double *in) {
	Grid *g = which_grid(S, which);
	if (!g->val) g->val = calloc(g->sizeProd[g->rank], sizeof(double));
	memcpy(g->val, in, g->sizeProd[g->rank] * sizeof(double));
	gSyncToDevice(g);
	return 0;
}

int pinc_sim_emigrants(PincSim *S, long *nEmigrants) {
	memcpy(nEmigrants, S->mpi->nEmigrants, S->mpi->nNeighbors * S->pop->nSpecies * sizeof(long));
	return 0;
}

int pinc_sim_species(PincSim *S, double *charge, double *mass) {
	memcpy(charge, S->pop->charge, S->pop->nSpecies * sizeof(double));
	memcpy(mass, S->pop->mass, S->pop->nSpecies * sizeof(double));
	return 0;
}

int pinc_sim_open_output(PincSim *S) {
	output_open(S);
	return 0;
}

int pinc_sim_write_output(PincSim *S, double n) {
	if (!S->output) output_open(S);
	output_write(S, n);
	return 0;
}

int pinc_sim_sync(PincSim *S) {
	(void)S;
	return pinc_hip_stream_sync(g_pinc.stream);
}

int pinc_sim_timers(PincSim *S, double *ms) {
	(void)S;
	pinc_phase_flush();
	for (int i = 0; i < PINC_NPHASES; i++) ms[i] = g_pinc.phaseMs[i];
	return 0;
}

int pinc_sim_timers_reset(PincSim *S) {
	(void)S;
	/* intervals still in flight are dropped with the totals */
	for (int i = 0; i < PINC_NPHASES; i++) {
		g_pinc.phaseMs[i] = 0;
		if (!g_pinc.phaseOpen[i]) g_pinc.phaseN[i] = 0;
	}
	return 0;
}
