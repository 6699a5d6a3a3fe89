/*
 * orc_sim.c -- TEST INFRASTRUCTURE (oracle).  The run-mode driver: restates
 * regular() of src/main.c:50-304 with the immersed-object hooks compiled
 * out (the object module does not compile), plus the
 * normalisation of src/units.c:61-252 it depends on.
 *
 *  ow_create     methods select + _set sanity (main.c:55-79, pusher.c:1047-
 *                1087), uAlloc/uNormalize, gAllocMpi (grid.c:502-545),
 *                pAlloc, gAlloc x4, mgAllocSolver, gCreateNeighborhood
 *  ow_init       pPosLattice, pVelZero|Maxwell, [pPosPerturb] (the
 *                reference has it commented out, main.c:152; Langmuir runs
 *                need it), extractEmigrants + puMigrate (main.c:145-157)
 *  ow_init_fields distr, FROMHALO add, solve, E=-grad phi, half-step acc
 *                (main.c:168-186)
 *  ow_step       one iteration of main.c:197-274.  Single-add by default;
 *                literal=1 reproduces main.c:231-235 (second FROMHALO add of
 *                rho and an extra solve).
 * The C entry points at the end (orc_*) are what tests/ load via ctypes.
 */
#include "orc.h"
#include <math.h>
#include <time.h>

/* per-rank loops run in parallel over the emulated ranks (OpenMP): every
 * rank's state is private to it and cross-rank combination happens after
 * the loop in rank order, so results are bit-identical to a serial run */
#define PER_RANK _Pragma("omp parallel for num_threads(orc_nthreads) schedule(static) if(w->P > 1)")

static double now_s(void){
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9*t.tv_nsec;
}

static const double elementaryCharge = 1.60217733e-19;
static const double electronMass = 9.10938188e-31;
static const double vacuumPermittivity = 8.854187817e-12;

/* --------------------------------------------------------------- units -- */
static void global_size(const OIni *ini, int nd, int *L, long *V){
	int *ts = oini_intarr(ini, "grid:trueSize", nd);
	int *ns = oini_intarr(ini, "grid:nSubdomains", nd);
	long v = 1;
	for(int d = 0; d < nd; d++){ L[d] = ns[d]*ts[d]; v *= L[d]; }
	*V = v;
	free(ts); free(ns);
}

static void units_normalize(OWorld *w){
	OIni *ini = w->ini;
	int nd = oini_int(ini, "grid:nDims");
	int ns = oini_int(ini, "population:nSpecies");
	/* parseIndirectInput (units.c:138-157) */
	int L[3]; long Vl;
	global_size(ini, nd, L, &Vl);
	double V = (double)Vl;
	double mul[3];
	for(int i = 0; i < nd; i++) mul[i] = 1.0/L[i];
	oini_applysuffix(ini, "population:nParticles", "pc", &V, 1);
	oini_applysuffix(ini, "population:nAlloc", "pc", &V, 1);
	oini_applysuffix(ini, "grid:nEmigrantsAlloc", "pc", &V, 1);
	oini_applysuffix(ini, "grid:stepSize", "tot", mul, nd);
	const char *method = oini_raw(ini, "methods:normalization");
	int semi = !strcmp(method, "semiSI");
	if(!semi && strcmp(method, "SI")) orc_die("methods:normalization not valid (must be SI or semiSI)");
	if(semi){ /* uSemiSI (units.c:159-189) */
		double *charge = oini_doublearr(ini, "population:charge", ns);
		double *mass = oini_doublearr(ini, "population:mass", ns);
		double *density = oini_doublearr(ini, "population:density", ns);
		double timeStep = oini_double(ini, "time:timeStep");
		if(fabs(charge[0]+1) > 1e-10) orc_die("Species 0 must have charge -1 with this normalization");
		if(fabs(mass[0]-1) > 1e-10) orc_die("Species 0 must have mass 1 with this normalization");
		for(int s = 0; s < ns; s++){ charge[s] *= elementaryCharge; mass[s] *= electronMass; }
		double wpe = sqrt(pow(elementaryCharge,2)*density[0]/(vacuumPermittivity*electronMass));
		timeStep /= wpe;
		oini_setdoublearr(ini, "population:charge", charge, ns);
		oini_setdoublearr(ini, "population:mass", mass, ns);
		oini_setdouble(ini, "time:timeStep", timeStep);
		free(charge); free(mass); free(density);
	}
	/* uSI (units.c:191-231) */
	double timeStep = oini_double(ini, "time:timeStep");
	double *stepSize = oini_doublearr(ini, "grid:stepSize", nd);
	long *nPart = oini_longarr(ini, "population:nParticles", ns);
	double *density = oini_doublearr(ini, "population:density", ns);
	double *charge = oini_doublearr(ini, "population:charge", ns);
	double Vol = (double)Vl*pow(stepSize[0], nd);
	for(int s = 0; s < ns; s++) w->weights[s] = density[s]*Vol/nPart[s];
	double X = stepSize[0], T = timeStep, Q = w->weights[0]*fabs(charge[0]);
	double M = pow(T*Q,2)/(vacuumPermittivity*pow(X,nd));
	w->unitLength = X; w->unitTime = T; w->unitCharge = Q; w->unitMass = M;
	free(stepSize); free(nPart); free(density); free(charge);
	/* derived units (units.c:233-252) */
	double velocity = X/T;
	double eField = X*M/(pow(T,2)*Q);
	double bField = M/(T*Q);
	double unitDensity = 1.0/pow(X, (double)nd);
	/* uNormalize (units.c:78-120) */
	double *c = oini_doublearr(ini, "population:charge", ns);
	double *m = oini_doublearr(ini, "population:mass", ns);
	double *dn = oini_doublearr(ini, "population:density", ns);
	for(int s = 0; s < ns; s++){ c[s] *= w->weights[s]; m[s] *= w->weights[s]; dn[s] /= w->weights[s]; }
	for(int s = 0; s < ns; s++){ c[s] *= 1.0/Q; m[s] *= 1.0/M; dn[s] *= 1.0/unitDensity; }
	oini_setdoublearr(ini, "population:charge", c, ns);
	oini_setdoublearr(ini, "population:mass", m, ns);
	oini_setdoublearr(ini, "population:density", dn, ns);
	free(c); free(m); free(dn);
	oini_scaledouble(ini, "population:thermalVelocity", 1.0/velocity);
	oini_scaledouble(ini, "population:drift", 1.0/velocity);
	oini_scaledouble(ini, "population:perturbAmplitude", 1.0/X);
	oini_scaledouble(ini, "fields:BExt", 1.0/bField);
	oini_scaledouble(ini, "fields:EExt", 1.0/eField);
}

/* ------------------------------------------------------------- selects -- */
static int pick(const OIni *ini, const char *key, const char **names, int n){
	const char *v = oini_raw(ini, key);
	for(int i = 0; i < n; i++) if(!strcmp(v, names[i])) return i;
	orc_die("%s=%s invalid", key, v);
	return -1;
}

static void sanity(const OIni *ini, int dim, int order){
	int nd = oini_int(ini, "grid:nDims");
	int *ng = oini_intarr(ini, "grid:nGhostLayers", 2*nd);
	double *th = oini_doublearr(ini, "grid:thresholds", 2*nd);
	int minL = ng[0];
	double mn = th[0], mx = th[0];
	for(int i = 1; i < 2*nd; i++){
		if(ng[i] < minL) minL = ng[i];
		if(th[i] < mn) mn = th[i];
		if(th[i] > mx) mx = th[i];
	}
	if(nd != dim && dim != 0) orc_die("operator only supports grid:nDims=%d", dim);
	if(minL < 1) orc_die("requires grid:nGhostLayers >= 1");
	double reqMin = order == 0 ? -0.5 : (order == 1 ? 0 : 0.5);
	if(mn < reqMin) orc_die("requires grid:thresholds >= %.1f", reqMin);
	if(mx > minL - 0.5) orc_die("requires grid:thresholds <= grid:nGhostLayers - 0.5");
	free(ng); free(th);
}

static void select_methods(OWorld *w){
	OIni *ini = w->ini;
	const char *acc[] = {"puAcc3D1KE", "puAccND1KE", "puAcc3D1", "puAccND1", "puBoris3D1KE", "puBoris3D1",
	                     "puAccND0KE", "puAccND0"};
	w->acc = pick(ini, "methods:acc", acc, 8);
	/* puAccND0_set returns puAccND0KE (pusher.c:356-358) */
	if(w->acc == ORC_ACC_ND0) w->acc = ORC_ACC_ND0KE;
	const int acc0 = w->acc == ORC_ACC_ND0KE;
	sanity(ini, (w->acc == ORC_ACC_ND1KE || w->acc == ORC_ACC_ND1 || acc0) ? 0 : 3, acc0 ? 0 : 1);
	const char *distr[] = {"puDistr3D1", "puDistrND1", "puDistrND0"};
	w->distr = pick(ini, "methods:distr", distr, 3);
	sanity(ini, w->distr == ORC_DISTR_3D1 ? 3 : 0, w->distr == ORC_DISTR_ND0 ? 0 : 1);
	const char *mig[] = {"puExtractEmigrants3D", "puExtractEmigrantsND"};
	w->migrate = pick(ini, "methods:migrate", mig, 2);
	if(w->migrate == ORC_MIG_3D && oini_int(ini, "grid:nDims") != 3)
		orc_die("puExtractEmigrants3D requires grid:nDims=3");
	const char *poi[] = {"mgSolver", "sSolver"};
	w->poisson = pick(ini, "methods:poisson", poi, 2);
	int nd = oini_int(ini, "grid:nDims");
	if(w->poisson == ORC_POISSON_MG){
		if(strcmp(oini_raw(ini, "multigrid:cycle"), "mgVRecursive"))
			orc_die("only multigrid:cycle=mgVRecursive is on the hot path");
		const char *sm[] = {"gaussSeidelRB", "gaussSeidelRBND"};
		int a = pick(ini, "multigrid:preSmooth", sm, 2);
		int b = pick(ini, "multigrid:postSmooth", sm, 2);
		int c = pick(ini, "multigrid:coarseSolver", sm, 2);
		int v[3] = {a, b, c};
		for(int i = 0; i < 3; i++){
			if(v[i] == 0 && nd != 3) orc_die("gaussSeidelRB is implemented for 3-D only");
			v[i] = v[i] == 0 ? ORC_SMOOTH_GS3D : ORC_SMOOTH_GSND;
		}
		w->preSmooth = v[0]; w->postSmooth = v[1]; w->coarseSolv = v[2];
		const char *re[] = {"halfWeight", "halfWeightND"};
		const char *pr[] = {"bilinear", "bilinearND"};
		int rr = pick(ini, "multigrid:restrictor", re, 2);
		int pp = pick(ini, "multigrid:prolongator", pr, 2);
		if((rr == 0 || pp == 0) && nd != 3) orc_die("halfWeight/bilinear are implemented for 3-D only");
		w->restrictor = rr == 0 ? ORC_RESTR_3D : ORC_RESTR_ND;
		w->prolongator = pp == 0 ? ORC_PROL_3D : ORC_PROL_ND;
		w->nLevels = oini_int(ini, "multigrid:mgLevels");
		w->mgCycles = oini_int(ini, "multigrid:mgCycles");
		w->nPre = oini_int(ini, "multigrid:nPreSmooth");
		w->nPost = oini_int(ini, "multigrid:nPostSmooth");
		w->nCoarse = oini_int(ini, "multigrid:nCoarseSolve");
		if(w->nLevels < 1) orc_die("Multi Grid levels is 0");
		if(!w->mgCycles) orc_die("MG cycles is 0");
	} else {
		/* spectral.c:80-89 restricts the solver to nDims=1 without
		 * decomposition; the build extends it to 1-3 dimensions and slabs
		 * (global transform), and so does this checker */
		if(nd < 1 || nd > 3) orc_die("sSolver supports grid:nDims=1..3");
	}
}

/* ------------------------------------------------------------- world -- */
OWorld *ow_create(OIni *ini, int literal){
	OWorld *w = calloc(1, sizeof(*w));
	{ const char *ev = getenv("ORC_VERBOSE"); w->verbose = ev ? atoi(ev) : 0; }
	{ const char *ev = getenv("ORC_THREADS"); if(ev && atoi(ev) > 0) orc_nthreads = atoi(ev); }
	w->ini = ini;
	w->literal = literal;
	select_methods(w);
	units_normalize(w);
	int nd = oini_int(ini, "grid:nDims");
	int ns = oini_int(ini, "population:nSpecies");
	if(w->acc == ORC_ACC_BORIS3D1KE || w->acc == ORC_ACC_BORIS3D1){
		/* puGet3DRotationParameters on the normalised ini (pusher.c:485-505) */
		if(ns > 8) orc_die("Boris: at most 8 species");
		double *B = oini_doublearr(ini, "fields:BExt", nd);
		double *c = oini_doublearr(ini, "population:charge", ns);
		double *m = oini_doublearr(ini, "population:mass", ns);
		opu_rotation_params(ns, B, c, m, w->borisT, w->borisS);
		free(B); free(c); free(m);
	}
	w->nDims = nd; w->nSpecies = ns;
	int *nsub = oini_intarr(ini, "grid:nSubdomains", nd);
	int *ng = oini_intarr(ini, "grid:nGhostLayers", 2*nd);
	int *ts = oini_intarr(ini, "grid:trueSize", nd);
	int P = 1;
	for(int d = 0; d < nd; d++) P *= nsub[d];
	w->P = P;
	w->r = calloc(P, sizeof(ORank));
	w->keSpecies = calloc(ns, sizeof(double));
	w->maxVel = oini_has(ini, "population:maxVel") ? oini_double(ini, "population:maxVel") : 1e300;
	for(int r = 0; r < P; r++){
		ORank *R = &w->r[r];
		OMpi *m = &R->mpi;
		m->mpiRank = r; m->mpiSize = P; m->nDims = nd; m->nSpecies = ns;
		m->nSubdomainsProd[0] = 1;
		int rr = r;
		for(int d = 0; d < nd; d++){
			m->nSubdomains[d] = nsub[d];
			m->nSubdomainsProd[d+1] = m->nSubdomainsProd[d]*nsub[d];
			m->subdomain[d] = rr % nsub[d];
			rr /= nsub[d];
			m->offset[d] = m->subdomain[d]*ts[d] - ng[d];
			m->posToSubdomain[d] = (double)1/ts[d];
		}
		op_alloc(&R->pop, ini, P);
		og_alloc(&R->E, ini, -1);
		og_alloc(&R->rho, ini, 1);
		og_alloc(&R->phi, ini, 1);
		og_alloc(&R->res, ini, 1);
		om_create_neighborhood(m, ini, &R->rho);
	}
	free(nsub); free(ng); free(ts);
	if(w->poisson == ORC_POISSON_MG) ow_mg_alloc(w);
	if(w->poisson == ORC_POISSON_MG && oini_has(ini, "multigrid:native") && oini_int(ini, "multigrid:native")){
		int Tg[3] = {1, 1, 1};
		for(int d = 0; d < nd; d++) Tg[d] = w->r[0].rho.trueSize[d+1]*w->r[0].mpi.nSubdomains[d];
		w->native = on_alloc(nd, Tg, w->nLevels, w->restrictor == ORC_RESTR_3D);
		/* multigrid:extrapolate, as pinc_mg.c */
		on_set_extrapolate(w->native, oini_has(ini, "multigrid:extrapolate") && oini_int(ini, "multigrid:extrapolate"),
		                   oini_has(ini, "objects:sphere") || oini_has(ini, "objects:file"));
		on_set_spectral_coarse(w->native, oini_has(ini, "multigrid:spectralCoarse") &&
		                                  oini_int(ini, "multigrid:spectralCoarse"));
		if(oini_has(ini, "objects:secondGuess")){
			on_set_second_spectral(w->native, !strcmp(oini_raw(ini, "objects:secondGuess"), "spectral"));
		}
	}
	else if(nd == 1 && w->P == 1){
		int N = w->r[0].rho.trueSize[1];
		int M = N/2 + 1;
		w->spectralFactor = calloc(M, sizeof(double));
		for(int n = 1; n < M; n++){
			double f = N/(2*M_PI*n);
			f *= f;
			f /= N;
			w->spectralFactor[n] = f;
		}
	}
	return w;
}

void ow_free(OWorld *w){
	for(int r = 0; r < w->P; r++){
		ORank *R = &w->r[r];
		op_free(&R->pop);
		og_free(&R->E); og_free(&R->rho); og_free(&R->phi); og_free(&R->res);
		OMg *m[3] = {&R->mgRho, &R->mgPhi, &R->mgRes};
		for(int k = 0; k < 3; k++){
			for(int q = 1; q < m[k]->nLevels; q++){ og_free(m[k]->grids[q]); free(m[k]->grids[q]); }
			free(m[k]->grids);
		}
		OMpi *mp = &R->mpi;
		for(int ne = 0; ne < mp->nNeighbors; ne++){ free(mp->emigrants[ne]); free(mp->emigrantIds[ne]); }
		free(mp->emigrants); free(mp->emigrantIds);
		free(mp->nEmigrants); free(mp->nImmigrants); free(mp->nEmigrantsAlloc);
	}
	free(w->r); free(w->keSpecies); free(w->spectralFactor); free(w->mgHist);
	on_free(w->native);
	oini_free(w->ini);
	free(w);
}

/* ---------------------------------------------------------- operators -- */
static void do_extract(OWorld *w){
	PER_RANK
	for(int r = 0; r < w->P; r++){
		if(w->migrate == ORC_MIG_3D) opu_extract3d(&w->r[r].pop, &w->r[r].mpi);
		else opu_extractnd(&w->r[r].pop, &w->r[r].mpi);
	}
}

static void do_distr(OWorld *w){
	OGrid *rho[256];
	PER_RANK
	for(int r = 0; r < w->P; r++){
		if(w->distr == ORC_DISTR_3D1) opu_distr3d1(&w->r[r].pop, &w->r[r].rho);
		else if(w->distr == ORC_DISTR_ND0) opu_distrnd0(&w->r[r].pop, &w->r[r].rho);
		else opu_distrnd1(&w->r[r].pop, &w->r[r].rho);
		rho[r] = &w->r[r].rho;
	}
	ow_halo(w, rho, OP_ADD, FROMHALO);
}

static void do_solve(OWorld *w){
	if(w->native) ow_native_solve(w);
	else if(w->poisson == ORC_POISSON_MG) ow_mg_solve(w);
	else ow_spectral_solve(w);
}

static void do_efield(OWorld *w, int haloPhi){
	OGrid *phi[256], *E[256];
	for(int r = 0; r < w->P; r++){ phi[r] = &w->r[r].phi; E[r] = &w->r[r].E; }
	if(haloPhi) ow_halo(w, phi, OP_SET, TOHALO);
	for(int r = 0; r < w->P; r++) og_findiff1st(phi[r], E[r]);
	ow_halo(w, E, OP_SET, TOHALO);
	for(int r = 0; r < w->P; r++) og_mul(E[r], -1.);
}

static void do_acc(OWorld *w){
	PER_RANK
	for(int r = 0; r < w->P; r++){
		OPop *p = &w->r[r].pop;
		OGrid *E = &w->r[r].E;
		switch(w->acc){
		case ORC_ACC_3D1KE: opu_acc3d1(p, E, 1); break;
		case ORC_ACC_3D1:   opu_acc3d1(p, E, 0); break;
		case ORC_ACC_ND1KE: opu_accnd1(p, E, 1); break;
		case ORC_ACC_BORIS3D1KE: opu_boris3d1(p, E, w->borisT, w->borisS, 1); break;
		case ORC_ACC_BORIS3D1:   opu_boris3d1(p, E, w->borisT, w->borisS, 0); break;
		case ORC_ACC_ND0KE: opu_accnd0(p, E, 1); break;
		default:            opu_accnd1(p, E, 0); break;
		}
	}
}

static void do_energy(OWorld *w){
	int ns = w->nSpecies;
	double ke = 0, pe = 0;
	for(int s = 0; s < ns; s++) w->keSpecies[s] = 0;
	PER_RANK
	for(int r = 0; r < w->P; r++){
		OPop *p = &w->r[r].pop;
		op_sum_kin(p);
		p->potEnergy[ns] = og_pot_energy_inner(&w->r[r].rho, &w->r[r].phi)*0.5;
	}
	for(int r = 0; r < w->P; r++){
		OPop *p = &w->r[r].pop;
		ke += p->kinEnergy[ns];
		for(int s = 0; s < ns; s++) w->keSpecies[s] += p->kinEnergy[s];
		pe += p->potEnergy[ns];
	}
	w->lastKE = ke;
	w->lastPE = pe;
}

void ow_init(OWorld *w, int perturb, int maxwell, unsigned long long seed){
	PER_RANK
	for(int r = 0; r < w->P; r++){
		ORank *R = &w->r[r];
		op_pos_lattice(&R->pop, w->ini, &R->mpi);
		if(maxwell) op_vel_maxwell(&R->pop, w->ini, seed);
		else op_vel_zero(&R->pop);
		if(perturb) op_pos_perturb(&R->pop, w->ini, &R->mpi);
	}
	do_extract(w);
	ow_migrate(w);
}

void ow_init_fields(OWorld *w){
	do_distr(w);
	do_solve(w);
	/* main.c:168-186 takes E from phi without a TOHALO.  After mgSolve the
	 * ghosts are valid (the smoother's halo exchanges); after sSolve they
	 * are stale (gInsertHalo, grid.c:892-915, does not refill them), so the
	 * reference's initial E is wrong at the edge nodes.  The build computes
	 * E from the periodic phi; the checker follows. */
	do_efield(w, w->poisson == ORC_POISSON_SPECTRAL);
	for(int r = 0; r < w->P; r++) og_mul(&w->r[r].E, 0.5);
	if(w->acc == ORC_ACC_BORIS3D1KE || w->acc == ORC_ACC_BORIS3D1){
		/* half step of the Boris extension: E and T halved, S for the halved
		 * T (pusher.h:66-70 documents halving E, S and T) */
		double T[24], S[24];
		memcpy(T, w->borisT, sizeof(T));
		memcpy(S, w->borisS, sizeof(S));
		for(int i = 0; i < 24; i += 3){
			double denom = 1;
			for(int q = 0; q < 3; q++){ w->borisT[i+q] = 0.5*T[i+q]; denom += w->borisT[i+q]*w->borisT[i+q]; }
			for(int q = 0; q < 3; q++) w->borisS[i+q] = 2.0/denom*w->borisT[i+q];
		}
		do_acc(w);
		memcpy(w->borisT, T, sizeof(T));
		memcpy(w->borisS, S, sizeof(S));
	} else {
		do_acc(w);
	}
	for(int r = 0; r < w->P; r++) og_mul(&w->r[r].E, 2.0);
}

void ow_step(OWorld *w){
	/* per-phase wall times: move, extract+migrate, deposit (+fold), solve,
	 * E field, accelerate, energies */
	double t0 = now_s(), t;
	PER_RANK
	for(int r = 0; r < w->P; r++) opu_move(&w->r[r].pop);
	t = now_s(); w->phaseT[0] += t - t0; t0 = t;
	do_extract(w);
	ow_migrate(w);
	t = now_s(); w->phaseT[1] += t - t0; t0 = t;
	do_distr(w);
	t = now_s(); w->phaseT[2] += t - t0; t0 = t;
	if(w->literal){
		OGrid *rho[256];
		for(int r = 0; r < w->P; r++) rho[r] = &w->r[r].rho;
		ow_halo(w, rho, OP_ADD, FROMHALO);
		do_solve(w);
	}
	do_solve(w);
	t = now_s(); w->phaseT[3] += t - t0; t0 = t;
	do_efield(w, 1);
	t = now_s(); w->phaseT[4] += t - t0; t0 = t;
	do_acc(w);
	t = now_s(); w->phaseT[5] += t - t0; t0 = t;
	do_energy(w);
	t = now_s(); w->phaseT[6] += t - t0;
}

/* main.c:197-274 with the immersed-object calls (main.c:221-238):
 * collect after migration, rho += rhoObj after the fold (the literal mode
 * folds again, main.c:232), solve, capacitance correction, solve again */
void oo_step(OWorld *w, OObj *o){
	if(w->P != 1) orc_die("object oracle: one subdomain only");
	opu_move(&w->r[0].pop);
	do_extract(w);
	ow_migrate(w);
	oo_collect(o, w);
	do_distr(w);
	og_addto(&w->r[0].rho, oo_rho_obj_grid(o));
	if(w->literal){
		OGrid *rho[1] = {&w->r[0].rho};
		ow_halo(w, rho, OP_ADD, FROMHALO);
	}
	if(w->native) on_guess_next(w->native, ON_GUESS_FIRST);
	do_solve(w);
	oo_apply(o, w, NULL);
	if(w->native) on_guess_next(w->native, ON_GUESS_SECOND);
	do_solve(w);
	do_efield(w, 1);
	do_acc(w);
	do_energy(w);
}

/* main.c:163-166: particles initially inside an object are removed and
 * their charge discarded */
void oo_init_collect(OObj *o, OWorld *w){
	oo_collect(o, w);
	og_zero((OGrid *)oo_rho_obj_grid(o));
}

/* ======================================================= ctypes API ===== */
OWorld *orc_world_new(const char *iniPath, int nOver, const char **over, int literal){
	OIni *ini = oini_load(iniPath);
	for(int i = 0; i < nOver; i++){
		char buf[1024];
		snprintf(buf, sizeof(buf), "%s", over[i]);
		char *eq = strchr(buf, '=');
		if(!eq) orc_die("override without '=': %s", over[i]);
		*eq = '\0';
		oini_set(ini, buf, eq + 1);
	}
	return ow_create(ini, literal);
}

void orc_world_free(OWorld *w){ ow_free(w); }
void orc_world_init(OWorld *w, int perturb, int maxwell, unsigned long long seed){ ow_init(w, perturb, maxwell, seed); }
void orc_world_init_fields(OWorld *w){ ow_init_fields(w); }
void orc_world_step(OWorld *w){ ow_step(w); }
int orc_world_nranks(const OWorld *w){ return w->P; }
long orc_world_cycles(const OWorld *w){ return w->cycles; }
long orc_world_solves(const OWorld *w){ return w->solves; }
void orc_world_energy(const OWorld *w, double *ke, double *pe, double *keSpecies){
	*ke = w->lastKE; *pe = w->lastPE;
	if(keSpecies) memcpy(keSpecies, w->keSpecies, w->nSpecies*sizeof(double));
}
void orc_world_units(const OWorld *w, double *out){
	out[0] = w->unitLength; out[1] = w->unitTime; out[2] = w->unitCharge; out[3] = w->unitMass;
	for(int s = 0; s < w->nSpecies; s++) out[4+s] = w->weights[s];
}
/* normalised charge/mass as stored in the Population */
void orc_world_species(const OWorld *w, double *charge, double *mass){
	memcpy(charge, w->r[0].pop.charge, w->nSpecies*sizeof(double));
	memcpy(mass, w->r[0].pop.mass, w->nSpecies*sizeof(double));
}
const char *orc_world_ini_get(const OWorld *w, const char *key){ return oini_raw(w->ini, key); }

/* phase-level operators for unit parity tests */
void orc_op(OWorld *w, const char *name){
	if(!strcmp(name, "move")) for(int r = 0; r < w->P; r++) opu_move(&w->r[r].pop);
	else if(!strcmp(name, "extract")) do_extract(w);
	else if(!strcmp(name, "migrate")) ow_migrate(w);
	else if(!strcmp(name, "distr")) do_distr(w);          /* deposit + FROMHALO add */
	else if(!strcmp(name, "distr_nohalo")){
		for(int r = 0; r < w->P; r++){
			if(w->distr == ORC_DISTR_3D1) opu_distr3d1(&w->r[r].pop, &w->r[r].rho);
			else if(w->distr == ORC_DISTR_ND0) opu_distrnd0(&w->r[r].pop, &w->r[r].rho);
			else opu_distrnd1(&w->r[r].pop, &w->r[r].rho);
		}
	}
	else if(!strcmp(name, "solve")) do_solve(w);
	else if(!strcmp(name, "efield")) do_efield(w, 1);
	else if(!strcmp(name, "acc")) do_acc(w);
	else if(!strcmp(name, "energy")) do_energy(w);
	else orc_die("unknown op %s", name);
}

static OGrid *grid_sel(OWorld *w, int r, int which, int level){
	ORank *R = &w->r[r];
	switch(which){
	case 0: return &R->rho;
	case 1: return &R->phi;
	case 2: return &R->E;
	case 3: return &R->res;
	case 4: return R->mgRho.grids[level];
	case 5: return R->mgPhi.grids[level];
	case 6: return R->mgRes.grids[level];
	}
	orc_die("bad grid selector");
	return NULL;
}

/* size[0..3] and total element count */
long orc_grid_shape(OWorld *w, int r, int which, int level, int *size){
	OGrid *g = grid_sel(w, r, which, level);
	for(int d = 0; d < 4; d++) size[d] = d < g->rank ? g->size[d] : 1;
	return g->sizeProd[g->rank];
}
void orc_grid_get(OWorld *w, int r, int which, int level, double *out){
	OGrid *g = grid_sel(w, r, which, level);
	memcpy(out, g->val, g->sizeProd[g->rank]*sizeof(double));
}
void orc_grid_set(OWorld *w, int r, int which, int level, const double *in){
	OGrid *g = grid_sel(w, r, which, level);
	memcpy(g->val, in, g->sizeProd[g->rank]*sizeof(double));
}

long orc_pop_count(OWorld *w, int r, int s){ return w->r[r].pop.iStop[s] - w->r[r].pop.iStart[s]; }
long orc_pop_capacity(OWorld *w, int r, int s){ return w->r[r].pop.iStart[s+1] - w->r[r].pop.iStart[s]; }
void orc_pop_get(OWorld *w, int r, int s, double *pos, double *vel, long *id){
	OPop *p = &w->r[r].pop;
	long n = p->iStop[s] - p->iStart[s], nd = p->nDims;
	if(pos) memcpy(pos, p->pos + nd*p->iStart[s], n*nd*sizeof(double));
	if(vel) memcpy(vel, p->vel + nd*p->iStart[s], n*nd*sizeof(double));
	if(id) memcpy(id, p->id + p->iStart[s], n*sizeof(long));
}
void orc_pop_set(OWorld *w, int r, int s, long n, const double *pos, const double *vel, const long *id){
	OPop *p = &w->r[r].pop;
	long nd = p->nDims;
	if(n > p->iStart[s+1] - p->iStart[s]) orc_die("orc_pop_set: capacity");
	memcpy(p->pos + nd*p->iStart[s], pos, n*nd*sizeof(double));
	memcpy(p->vel + nd*p->iStart[s], vel, n*nd*sizeof(double));
	if(id) memcpy(p->id + p->iStart[s], id, n*sizeof(long));
	p->iStop[s] = p->iStart[s] + n;
}
void orc_pop_kinetic(OWorld *w, int r, double *ke){
	memcpy(ke, w->r[r].pop.kinEnergy, (w->nSpecies+1)*sizeof(double));
}
void orc_mpi_emigrants(OWorld *w, int r, long *nEmigrants){
	OMpi *m = &w->r[r].mpi;
	memcpy(nEmigrants, m->nEmigrants, m->nNeighbors*w->nSpecies*sizeof(long));
}
/* emigrants[ne] of the last extraction (pusher.c:827-833 layout: pos then
 * vel, nDims each, species after species): the number of records */
long orc_mpi_emigrant_buffer(OWorld *w, int r, int ne, double *out){
	OMpi *m = &w->r[r].mpi;
	if(ne < 0 || ne >= m->nNeighbors || ne == m->center) return 0;
	long cnt = 0;
	for(int s = 0; s < w->nSpecies; s++) cnt += m->nEmigrants[ne*w->nSpecies + s];
	if(out) memcpy(out, m->emigrants[ne], 2*w->nDims*cnt*sizeof(double));
	return cnt;
}
void orc_mpi_thresholds(OWorld *w, int r, double *thr){
	memcpy(thr, w->r[r].mpi.thresholds, 2*w->nDims*sizeof(double));
}
void orc_mpi_alloc(OWorld *w, int r, long *alloc){
	OMpi *m = &w->r[r].mpi;
	memcpy(alloc, m->nEmigrantsAlloc, m->nNeighbors*sizeof(long));
}

/* -------------------------------------------- known-answer test hooks -- */
/* Interpolate+accelerate on a bare grid (no ini): E has nDims components. */
void orc_kat_acc(int nd, const int *trueSize, int nGhost, double *Eval, long n,
                 const double *pos, double *vel, double charge, double mass, int use3d, double *ke){
	OGrid E; memset(&E, 0, sizeof(E));
	E.rank = nd + 1;
	E.size[0] = E.trueSize[0] = nd;
	for(int d = 1; d <= nd; d++){
		E.trueSize[d] = trueSize[d-1];
		E.nGhost[d] = E.nGhost[d+E.rank] = nGhost;
		E.size[d] = trueSize[d-1] + 2*nGhost;
	}
	E.sizeProd[0] = 1;
	for(int d = 0; d < E.rank; d++) E.sizeProd[d+1] = E.sizeProd[d]*E.size[d];
	E.val = Eval;
	OPop p; memset(&p, 0, sizeof(p));
	long iStart[2] = {0, n}, iStop[1] = {n};
	double q[1] = {charge}, m[1] = {mass}, kin[2] = {0, 0};
	p.nDims = nd; p.nSpecies = 1; p.iStart = iStart; p.iStop = iStop;
	p.pos = (double*)pos; p.vel = vel; p.charge = q; p.mass = m; p.kinEnergy = kin;
	if(use3d) opu_acc3d1(&p, &E, 1); else opu_accnd1(&p, &E, 1);
	if(ke) *ke = kin[0];
}

void orc_kat_distr(int nd, const int *trueSize, int nGhost, double *rhoval, long n,
                   const double *pos, double charge, int use3d){
	OGrid g; memset(&g, 0, sizeof(g));
	g.rank = nd + 1;
	g.size[0] = g.trueSize[0] = 1;
	for(int d = 1; d <= nd; d++){
		g.trueSize[d] = trueSize[d-1];
		g.nGhost[d] = g.nGhost[d+g.rank] = nGhost;
		g.size[d] = trueSize[d-1] + 2*nGhost;
	}
	g.sizeProd[0] = 1;
	for(int d = 0; d < g.rank; d++) g.sizeProd[d+1] = g.sizeProd[d]*g.size[d];
	g.val = rhoval;
	OPop p; memset(&p, 0, sizeof(p));
	long iStart[2] = {0, n}, iStop[1] = {n};
	double q[1] = {charge};
	p.nDims = nd; p.nSpecies = 1; p.iStart = iStart; p.iStop = iStop;
	p.pos = (double*)pos; p.charge = q;
	if(use3d) opu_distr3d1(&p, &g); else opu_distrnd1(&p, &g);
}

int orc_kat_neighbor_to_rank(const int *nSub, const int *sub, int neighbor){
	OMpi m; memset(&m, 0, sizeof(m));
	m.nDims = 3;
	m.nSubdomainsProd[0] = 1;
	for(int d = 0; d < 3; d++){
		m.nSubdomains[d] = nSub[d]; m.subdomain[d] = sub[d];
		m.nSubdomainsProd[d+1] = m.nSubdomainsProd[d]*nSub[d];
	}
	return opu_neighbor_to_rank(&m, neighbor);
}
int orc_kat_rank_to_neighbor(const int *nSub, const int *sub, int rank){
	OMpi m; memset(&m, 0, sizeof(m));
	m.nDims = 3;
	m.nSubdomainsProd[0] = 1;
	for(int d = 0; d < 3; d++){
		m.nSubdomains[d] = nSub[d]; m.subdomain[d] = sub[d];
		m.nSubdomainsProd[d+1] = m.nSubdomainsProd[d]*nSub[d];
	}
	return opu_rank_to_neighbor(&m, rank);
}
int orc_kat_reciprocal(int neighbor, int nDims){ return opu_neighbor_to_reciprocal(neighbor, nDims); }

/* thresholds / emigrant buffer sizes from an ini text (grid.c:1029-1132) */
void orc_kat_neighborhood(const char *iniText, double *thr, long *alloc){
	OIni *ini = oini_from_string(iniText);
	OGrid g;
	og_alloc(&g, ini, 1);
	OMpi m; memset(&m, 0, sizeof(m));
	m.nDims = oini_int(ini, "grid:nDims");
	m.nSpecies = 1;
	om_create_neighborhood(&m, ini, &g);
	memcpy(thr, m.thresholds, 2*m.nDims*sizeof(double));
	memcpy(alloc, m.nEmigrantsAlloc, m.nNeighbors*sizeof(long));
	og_free(&g);
	oini_free(ini);
}

/* testExtractEmigrantsXD (test/pusher.test.c:360-545): the neighbourhood of
 * the ini text (gCreateNeighborhood, thresholds by the current rule), then
 * opu_extract3d (use3d) or opu_extractnd on the given AoS particles; no
 * operator selection (the test selects none, so puSanity's threshold bound
 * does not apply).  pos/vel/iStop are updated in place; nEmigrants gets the
 * nNeighbors*nSpecies counts, bufs the nNeighbors buffers of cap records
 * (2*nDims doubles each), thr the thresholds. */
void orc_kat_extract(const char *iniText, int nSpecies, const long *iStart, long *iStop, double *pos, double *vel,
                     int use3d, long *nEmigrants, double *bufs, long cap, double *thr){
	OIni *ini = oini_from_string(iniText);
	OGrid g;
	og_alloc(&g, ini, 1);
	OMpi m; memset(&m, 0, sizeof(m));
	m.nDims = oini_int(ini, "grid:nDims");
	m.nSpecies = nSpecies;
	om_create_neighborhood(&m, ini, &g);
	const int nd = m.nDims;
	OPop p; memset(&p, 0, sizeof(p));
	p.nDims = nd; p.nSpecies = nSpecies;
	p.iStart = (long*)iStart; p.iStop = iStop; p.pos = pos; p.vel = vel;
	p.id = calloc(iStart[nSpecies], sizeof(long));
	if(use3d) opu_extract3d(&p, &m); else opu_extractnd(&p, &m);
	memcpy(nEmigrants, m.nEmigrants, m.nNeighbors*nSpecies*sizeof(long));
	memcpy(thr, m.thresholds, 2*nd*sizeof(double));
	for(int ne = 0; ne < m.nNeighbors; ne++){
		if(ne == m.center) continue;
		long cnt = 0;
		for(int s = 0; s < nSpecies; s++) cnt += m.nEmigrants[ne*nSpecies + s];
		if(cnt > cap) orc_die("orc_kat_extract: %ld records for direction %d, cap %ld", cnt, ne, cap);
		memcpy(bufs + (long)ne*cap*2*nd, m.emigrants[ne], cnt*2*nd*sizeof(double));
		free(m.emigrants[ne]);
		free(m.emigrantIds[ne]);
	}
	free(m.emigrants); free(m.emigrantIds); free(m.nEmigrants); free(m.nImmigrants); free(m.nEmigrantsAlloc);
	free(p.id);
	og_free(&g);
	oini_free(ini);
}

int orc_world_ndims(const OWorld *w){ return w->nDims; }

/* multigrid diagnostics: cycles per solve (0 = until converged) and the
 * per-cycle RMS residual of the last solve */
void orc_world_mg_limit(OWorld *w, long maxCycles, long histCap){
	w->mgCap = maxCycles > 0 ? maxCycles : 0;
	free(w->mgHist);
	w->mgHist = histCap > 0 ? calloc(histCap, sizeof(double)) : NULL;
	w->mgHistCap = histCap > 0 ? histCap : 0;
	w->mgHistN = 0;
}
long orc_world_mg_history(const OWorld *w, double *out, long cap){
	long n = w->mgHistN < w->mgHistCap ? w->mgHistN : w->mgHistCap;
	if(out) for(long i = 0; i < n && i < cap; i++) out[i] = w->mgHist[i];
	return w->mgHistN;
}
void orc_set_threads(int n){ if(n > 0) orc_nthreads = n; }
/* seconds per phase since creation (see ow_step) */
void orc_world_timers(const OWorld *w, double *out){ memcpy(out, w->phaseT, 7*sizeof(double)); }
int orc_world_mg_levels(const OWorld *w){ return w->native ? on_levels(w->native) : w->nLevels; }
int orc_world_nspecies(const OWorld *w){ return w->nSpecies; }
