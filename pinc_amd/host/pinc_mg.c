/*
 * pinc_mg.c -- multigrid Poisson solver of the MI355X PINC hot path (host C).
 *
 * Parity mode (default) runs the reference algorithm of src/multigrid.c:
 *   mgAllocSolver      multigrid.c:364-384, levels T/2^q (mgAllocSubGrids 128-214)
 *   mgSolve/mgSolveRaw multigrid.c:403-407, 1688-1724: V-cycles until the RMS
 *                      residual over true nodes is <= 1e-10 (at least one)
 *   vrec               mgVRecursiveInner 1496-1556: neutralise rho, presmooth,
 *                      residual, restrict, recurse, add the prolongated
 *                      correction, neutralise, postsmooth, neutralise
 *   smoothers          mgGS3D / mgGSND red-black Gauss-Seidel with a
 *                      neutralisation after every colour (gBnd -> grid.c:730)
 * Coarse-level potentials persist between cycles and steps (warm start) as in
 * the reference.  The solve runs on the whole periodic domain on every rank:
 * with several ranks the slabs of rho are all-gathered first (RCCL) and every
 * rank computes the same potential, replacing the reference's per-colour
 * halo exchanges (DESIGN.md "Multi-GPU").
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>
#include <stdint.h>

#define MU_SLOT 32   /* two alternating mean slots of the smoother */
#define TMP_SLOT 40

void mgSolver(void (**solve)(), void *(**solverAlloc)(), void (**solverFree)()) {
	*solve = (void (*)())mgSolve;
	*solverAlloc = (void *(*)())mgAllocSolver;
	*solverFree = (void (*)())mgFreeSolver;
}

funPtr mgSolver_set(dictionary *ini) {
	(void)ini;
	return (funPtr)mgSolver;
}

static int smootherIs3D(const dictionary *ini, const char *key, int nd) {
	char *v = iniGetStr(ini, key);
	int r = -1;
	if (!strcmp(v, "gaussSeidelRB")) {
		if (nd != 3) msg(ERROR, "%s=gaussSeidelRB is 2-D/3-D specific; the device path implements 3-D (use gaussSeidelRBND)", key);
		r = 1;
	} else if (!strcmp(v, "gaussSeidelRBND")) r = 0;
	else msg(ERROR, "%s=%s is not on the MI355X hot path", key, v);
	free(v);
	return r;
}

/* Sharded level 0 (native mode).  multigrid:shard = 0
 * (replicated solve), 1 (shard whenever the geometry allows it, also on one
 * rank, whose halo is then its own periodic image) or auto (default: shard
 * with several ranks once the extended slab is at most half the global
 * grid, i.e. from 4 ranks at 256^3).  Each rank smooths its z-slab extended
 * by hz planes on each side; after `chunk` red-black iterations the planes
 * within 2 chunk + 2 of the slab ends are stale, so the halo is refreshed
 * (hz planes each way) before every chunk, and hz >= 2 chunk + 2 keeps the
 * planes that the residual, the restriction and E read exact. */
static void shard_setup(MultigridSolver *S, const dictionary *ini, const Grid *rho, Grid *phi) {
	pinc_geom_t g = rho->dev->geom;
	int mode = -1; /* auto */
	if (iniHas(ini, "multigrid:shard")) {
		char *v = iniGetStr(ini, "multigrid:shard");
		if (!strcmp(v, "auto")) mode = -1;
		else mode = atoi(v) ? 1 : 0;
		free(v);
	}
	S->shard = 0;
	int nl = g.nloc;
	int m = S->nPre > S->nPost ? S->nPre : S->nPost;
	if (m > (nl - 2) / 2) m = (nl - 2) / 2;
	/* (objects shard too: pinc_obj.c reads the surface potentials from the
	 * slabs and sums them over the ranks, object.c:163-364's MPI pattern) */
	int ok = S->native && g.nd == 3 && S->nLevels >= 2 && nl % 2 == 0 && m >= 1;
	if (!mode || !ok) {
		if (mode == 1 && !ok)
			msg(WARNING, "multigrid:shard=1 needs native mode, 3-D and slabs of >= 4 planes: replicated solve");
		return;
	}
	int h = 2 * m + 2;
	/* extended slab a multiple of 16 planes (the fused sweeps), if the slab
	 * is deep enough to supply the extra halo */
	for (int h2 = h; h2 <= nl; h2 += 2)
		if ((nl + 2 * h2) % 16 == 0) {
			h = h2;
			break;
		}
	int E = nl + 2 * h;
	if (mode < 0 && !(g_pinc.nranks > 1 && 2 * E <= g.T[2])) return;
	S->shard = 1;
	S->hz = h;
	S->chunk = m;
	S->nloc0 = nl;
	S->ps0 = (long)g.T[0] * g.T[1];
	S->z0 = g.off - h;
	S->L[0].T[2] = E;
	S->N[0] = S->ps0 * E;
	S->L1s = S->L[1];
	S->L1s.T[2] = nl / 2;
	long n1 = (long)S->L1s.T[0] * S->L1s.T[1] * S->L1s.T[2];
	pinc_check(pinc_hip_malloc((void **)&S->rho1Slab, n1 * sizeof(double)), "mg shard");
	/* rho[0], phi[0], res[0] are allocated with the other levels (size N[0]) */
	phi->dev->extOff = h;
	phi->dev->extPlanes = E;
	S->useGraph = 0; /* the halo exchanges are host-driven */
}

enum { kSmallOut = 64, kSmallHist = 60, kSmallChunk = 1000 };

/* native mode, one rank, a 2-D level 0 of at most 16384 points (a multiple
 * of 2048) with a power-of-two x extent <= 1024, its levels 1.. within the
 * one-workgroup coarse solve's LDS budget: the whole solve in one launch per
 * solve (pinc_hip_mg_solve_small).  multigrid:oneCU (default 0) or
 * PINC_MG_SMALL (experiments) turn it on.  With multigrid:spectralCoarse the
 * workgroup solves level 1 exactly itself (no rocFFT plan is made). */
static int small_eligible(const MultigridSolver *S, const dictionary *ini) {
	int want = iniHas(ini, "multigrid:oneCU") && iniGetInt(ini, "multigrid:oneCU");
	if (getenv("PINC_MG_SMALL")) want = atoi(getenv("PINC_MG_SMALL"));
	if (!want || !S->native || S->shard || g_pinc.nranks != 1 || S->nLevels < 2) return 0;
	const pinc_lvl_t L = S->L[0];
	const long n0 = (long)L.T[0] * L.T[1];
	if (L.nd != 2 || (L.T[0] & (L.T[0] - 1)) || L.T[0] < 2 || L.T[0] > 1024 || L.T[1] % 2 || n0 > 16384 || n0 % 2048)
		return 0;
	long tot = 0;
	for (int q = 1; q < S->nLevels; q++) tot += 3 * S->N[q];
	return tot <= 5500 * 3 && S->nLevels - 1 <= 12;
}

/* level 1's real orthonormal Fourier basis for the workgroup's exact
 * coarse solve (pinc_hip_mg_solve_small): Q[j][k] = DC 1/sqrt(n) (k = 0),
 * sqrt(2/n) cos(2 pi j k / n) (0 < k < n/2), Nyquist (-1)^j / sqrt(n)
 * (k = n/2), sqrt(2/n) sin(2 pi j (k - n/2) / n) (k > n/2); then the
 * eigenvalue 2 - 2 cos(2 pi f / n) of each column (k_spectral_scale's
 * symbol, per dimension) */
static void small_basis(MultigridSolver *S, int n) {
	double *h = malloc((size_t)(n * n + n) * sizeof(double));
	const int hn = n / 2;
	for (int j = 0; j < n; j++)
		for (int k = 0; k < n; k++) {
			double v;
			if (k == 0) v = 1.0 / sqrt((double)n);
			else if (k < hn) v = sqrt(2.0 / n) * cos(2 * M_PI * (double)((long)j * k % n) / n);
			else if (k == hn) v = (j & 1 ? -1.0 : 1.0) / sqrt((double)n);
			else v = sqrt(2.0 / n) * sin(2 * M_PI * (double)((long)j * (k - hn) % n) / n);
			h[j * n + k] = v;
		}
	for (int k = 0; k < n; k++) {
		const int f = k <= hn ? k : k - hn;
		h[n * n + k] = 2.0 - 2.0 * cos(2 * M_PI * f / n);
	}
	pinc_check(pinc_hip_malloc((void **)&S->smallBasis, (size_t)(n * n + n) * sizeof(double)), "mg small basis");
	pinc_check(pinc_hip_h2d(S->smallBasis, h, (size_t)(n * n + n) * sizeof(double), g_pinc.stream), "mg small basis");
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), "mg small basis");
	free(h);
}

/* the V-cycles of one solve in launches of at most kSmallChunk cycles (at
 * most kSmallHist when a history is kept), until the RMS residual is at most
 * 1e-10 as mgSolve's loop; returns the cycles run */
static long small_solve(MultigridSolver *S, long cap, double *lastRes) {
	long c = 0;
	double barRes = 2.;
	for (;;) {
		long chunk = S->histCap > 0 ? kSmallHist : kSmallChunk;
		if (cap > 0 && cap - c < chunk) chunk = cap - c;
		int slot = pinc_probe_begin(PINC_PROBE_CYCLE);
		pinc_check(pinc_hip_mg_solve_small(S->phi[0], S->rho[0], S->res[0], S->nLevels, S->L, S->nPre, S->nPost,
		                                   S->nCoarse, (int)chunk, 1.E-10, S->smallBasis, S->smallOut, g_pinc.stream),
		           "mg small solve");
		pinc_probe_end(PINC_PROBE_CYCLE, slot, 0.0);
		pinc_check(pinc_hip_d2h(S->hostSmall, S->smallOut, kSmallOut * sizeof(double), g_pinc.stream), "mg small solve");
		const long n = (long)S->hostSmall[0];
		barRes = S->hostSmall[1];
		for (long k = 0; k < n; k++) {
			if (S->histN < S->histCap) S->hist[S->histN] = k < kSmallHist ? S->hostSmall[2 + k] : NAN;
			S->histN++;
			if (g_pinc.verbose && ((c + k + 1) % g_pinc.verbose == 0) && k < kSmallHist) {
				fprintf(stderr, "[pinc] rank %d solve cycle %ld residual %.3e\n", g_pinc.rank, c + k + 1,
				        S->hostSmall[2 + k]);
				fflush(stderr);
			}
		}
		c += n;
		S->cycles += n;
		if (!(barRes > 1.E-10) || !isfinite(barRes) || (cap > 0 && c >= cap)) break;
		if (c > 1000000) break;
	}
	*lastRes = barRes;
	return c;
}

MultigridSolver *mgAllocSolver(const dictionary *ini, Grid *rho, Grid *phi) {
	MultigridSolver *S = calloc(1, sizeof(*S));
	int nd = rho->rank - 1;
	char *cycle = iniGetStr(ini, "multigrid:cycle");
	if (strcmp(cycle, "mgVRecursive")) msg(ERROR, "multigrid:cycle=%s: only mgVRecursive is on the hot path", cycle);
	free(cycle);
	S->nLevels = iniGetInt(ini, "multigrid:mgLevels");
	S->mgCycles = iniGetInt(ini, "multigrid:mgCycles");
	S->nPre = iniGetInt(ini, "multigrid:nPreSmooth");
	S->nPost = iniGetInt(ini, "multigrid:nPostSmooth");
	S->nCoarse = iniGetInt(ini, "multigrid:nCoarseSolve");
	if (S->nLevels < 1) msg(ERROR, "Multi Grid levels is 0, need 1 grid level");
	if (S->nLevels > PINC_MAX_LEVELS) msg(ERROR, "multigrid:mgLevels > %d", PINC_MAX_LEVELS);
	if (!S->mgCycles) msg(ERROR, "MG cycles is 0");
	S->pre3d = smootherIs3D(ini, "multigrid:preSmooth", nd);
	S->post3d = smootherIs3D(ini, "multigrid:postSmooth", nd);
	S->coarse3d = smootherIs3D(ini, "multigrid:coarseSolver", nd);
	char *re = iniGetStr(ini, "multigrid:restrictor");
	char *pr = iniGetStr(ini, "multigrid:prolongator");
	if (!strcmp(re, "halfWeight")) {
		if (nd != 3) msg(ERROR, "halfWeight is implemented for 3-D on the device path (use halfWeightND)");
		S->restr3d = 1;
	} else if (!strcmp(re, "halfWeightND")) S->restr3d = 0;
	else msg(ERROR, "multigrid:restrictor=%s not supported", re);
	if (strcmp(pr, "bilinear") && strcmp(pr, "bilinearND")) msg(ERROR, "multigrid:prolongator=%s not supported", pr);
	if (!strcmp(pr, "bilinear") && nd != 3) msg(ERROR, "bilinear is implemented for 3-D on the device path (use bilinearND)");
	free(re);
	free(pr);
	S->native = iniHas(ini, "multigrid:native") ? iniGetInt(ini, "multigrid:native") : 0;
	/* graph replay of the V-cycle (native mode, opt-in: measured neutral at
	 * C4, the gaps between dependent kernels are GPU-side) */
	S->useGraph = S->native && iniHas(ini, "multigrid:graph") && iniGetInt(ini, "multigrid:graph");
	S->cycleGraph = NULL;
	/* initial guesses extrapolated from earlier solutions (native mode,
	 * opt-in; guess_begin) */
	S->extrap = S->native && iniHas(ini, "multigrid:extrapolate") && iniGetInt(ini, "multigrid:extrapolate");
	S->objects = iniHas(ini, "objects:sphere") || iniHas(ini, "objects:file");
	S->havePrev = S->haveCorr = 0;
	S->role = S->objects ? PINC_MG_GUESS_WARM : PINC_MG_GUESS_SERIES;
	S->phiPrev = S->phiA = S->phiB = S->dCorr = NULL;
	S->secondSpectral = 0;
	S->rhoSave = S->dphi = NULL;
	S->fft = NULL;
	/* native mode: levels of at least fusedMin points smooth with the
	 * z-marching fused sweeps (two iterations per launch), smaller ones
	 * colour by colour (PINC_MG_FUSED_MIN overrides, experiments) */
	S->fusedMin = getenv("PINC_MG_FUSED_MIN") ? atol(getenv("PINC_MG_FUSED_MIN")) : (1L << 23);
	for (int d = 1; d <= nd; d++)
		if (rho->trueSize[d] % (1 << S->nLevels))
			msg(ERROR, "All elements in grid:trueSize must be a multiple of 2^mgLevels=%d", 1 << S->nLevels);
	pinc_geom_t g = rho->dev->geom;
	if (S->native) {
		/* native mode coarsens on down to 2 points per dimension, so the
		 * bottom solve is exact enough not to limit the cycle's convergence */
		for (;;) {
			int ok = S->nLevels < PINC_MAX_LEVELS;
			for (int d = 0; d < nd && ok; d++) {
				int t = g.T[d] >> (S->nLevels - 1);
				ok = (t % 2 == 0) && t / 2 >= 2;
			}
			if (!ok) break;
			S->nLevels++;
		}
	}
	for (int q = 0; q < S->nLevels; q++) {
		S->L[q].nd = nd;
		S->N[q] = 1;
		for (int d = 0; d < 3; d++) {
			S->L[q].T[d] = d < nd ? g.T[d] >> q : 1;
			S->N[q] *= S->L[q].T[d];
		}
	}
	long ps = rho->dev->planeSize;
	S->Ng0 = S->N[0];
	shard_setup(S, ini, rho, phi);
	if (S->shard) {
		/* level 0 is this rank's extended slab; no global level-0 arrays */
	} else if (g_pinc.nranks == 1) {
		rho->dev->global = rho->dev->d + ps;
		phi->dev->global = phi->dev->d + ps;
		phi->dev->globalIsTruth = 1;
	} else {
		pinc_check(pinc_hip_malloc((void **)&rho->dev->global, S->N[0] * sizeof(double)), "global rho");
		pinc_check(pinc_hip_malloc((void **)&phi->dev->global, S->N[0] * sizeof(double)), "global phi");
		pinc_check(pinc_hip_memset(phi->dev->global, 0, S->N[0] * sizeof(double), g_pinc.stream), "global phi");
		rho->dev->ownsGlobal = phi->dev->ownsGlobal = 1;
		phi->dev->globalIsTruth = 1;
	}
	if (!S->shard) {
		S->rho[0] = rho->dev->global;
		S->phi[0] = phi->dev->global;
	}
	for (int q = 0; q < S->nLevels; q++) {
		if (q > 0 || S->shard) {
			pinc_check(pinc_hip_malloc((void **)&S->rho[q], S->N[q] * sizeof(double)), "mg level");
			pinc_check(pinc_hip_malloc((void **)&S->phi[q], S->N[q] * sizeof(double)), "mg level");
			pinc_check(pinc_hip_memset(S->rho[q], 0, S->N[q] * sizeof(double), g_pinc.stream), "mg level");
			pinc_check(pinc_hip_memset(S->phi[q], 0, S->N[q] * sizeof(double), g_pinc.stream), "mg level");
		}
		pinc_check(pinc_hip_malloc((void **)&S->res[q], S->N[q] * sizeof(double)), "mg level");
	}
	if (S->shard) phi->dev->ext = S->phi[0];
	if (S->extrap && !S->objects)
		pinc_check(pinc_hip_malloc((void **)&S->phiPrev, S->N[0] * sizeof(double)), "mg extrapolation");
	if (S->extrap && S->objects && iniHas(ini, "objects:secondGuess")) {
		char *v = iniGetStr(ini, "objects:secondGuess");
		/* replicated solve: rho[0] and phi[0] global on every rank (rho[0]
		 * gathered before guess_begin), one transform of the global grid;
		 * sharded level 0: the owned planes, a slab-distributed transform */
		if (!strcmp(v, "spectral")) {
			if (!S->shard) S->secondSpectral = 1;
			else if (g.T[1] % g_pinc.nranks == 0 && g.T[2] == g.nloc * g_pinc.nranks) S->secondSpectral = 2;
			else msg(WARNING, "objects:secondGuess = spectral on the sharded solve needs grid:trueSize y divisible by "
			                  "the rank count: the last correction response instead");
		} else if (strcmp(v, "response")) msg(ERROR, "objects:secondGuess = %s (spectral | response)", v);
		free(v);
	}
	/* (PINC_MG_SPECULATE=0 overrides the ini: A/B runs of the bench) */
	S->speculate = S->native && !S->shard && !S->useGraph && S->nLevels > 1 &&
	               (!iniHas(ini, "multigrid:speculate") || iniGetInt(ini, "multigrid:speculate")) &&
	               !(getenv("PINC_MG_SPECULATE") && !atoi(getenv("PINC_MG_SPECULATE")));
	/* the norm is read into pinned memory (no staging copy on the host's
	 * wake-up path), with an event when speculating */
	pinc_check(pinc_hip_host_alloc((void **)&S->hostNorm, sizeof(double)), "mg norm");
	if (S->speculate) pinc_check(pinc_hip_event_create(&S->normEvent), "mg norm");
	S->small = small_eligible(S, ini);
	if (S->small && iniHas(ini, "multigrid:spectralCoarse") && iniGetInt(ini, "multigrid:spectralCoarse")) {
		/* the two-grid cycle in the workgroup: level 1 square, n = 16..64 in
		 * 16s (otherwise the per-level launches with rocFFT) */
		const int n = S->L[1].T[0];
		if (S->L[1].T[1] == n && n % 16 == 0 && n <= 64) small_basis(S, n);
		else S->small = 0;
	}
	if (S->small) {
		pinc_check(pinc_hip_malloc((void **)&S->smallOut, kSmallOut * sizeof(double)), "mg small solve");
		pinc_check(pinc_hip_host_alloc((void **)&S->hostSmall, kSmallOut * sizeof(double)), "mg small solve");
	}
	if (S->native && S->nLevels >= 2 && !S->small && iniHas(ini, "multigrid:spectralCoarse") &&
	    iniGetInt(ini, "multigrid:spectralCoarse")) {
		/* sharded level 0: level 1 stays decomposed when its slabs can be
		 * transposed (y divisible by the rank count), as the reference keeps
		 * every level on its subdomain (multigrid.c:128-180); PINC_MG_DIST1=0
		 * all-gathers it instead (the round-5 form) */
		const int n1 = S->shard ? S->nloc0 / 2 : 0;
		if (S->shard && n1 >= 1 && S->L[1].T[1] % g_pinc.nranks == 0 && S->L[1].T[2] == n1 * g_pinc.nranks &&
		    !(getenv("PINC_MG_DIST1") && !atoi(getenv("PINC_MG_DIST1")))) {
			S->dist1 = 1;
			pinc_check(pinc_hip_fft_slab_create(&S->fftCoarseSlab, S->L[1].T, n1, g_pinc.nranks, g_pinc.rank,
			                                    g_pinc.stream),
			           "mg spectral coarse (slabs)");
			pinc_check(pinc_hip_fft_slab_set_symbol(S->fftCoarseSlab, 1), "mg spectral coarse (slabs)");
			const long ps1 = (long)S->L[1].T[0] * S->L[1].T[1];
			pinc_check(pinc_hip_malloc((void **)&S->phi1Ext, ps1 * (n1 + 2) * sizeof(double)), "mg level 1 slab");
			pinc_check(pinc_hip_memset(S->phi1Ext, 0, ps1 * (n1 + 2) * sizeof(double), g_pinc.stream),
			           "mg level 1 slab");
		} else {
			pinc_check(pinc_hip_fft_create(&S->fftCoarse, S->L[1].nd, S->L[1].T, g_pinc.stream), "mg spectral coarse");
			pinc_check(pinc_hip_fft_set_symbol(S->fftCoarse, 1), "mg spectral coarse");
		}
	}
	if (S->secondSpectral == 1) {
		pinc_check(pinc_hip_malloc((void **)&S->rhoSave, S->N[0] * sizeof(double)), "mg second guess");
		pinc_check(pinc_hip_malloc((void **)&S->dphi, S->N[0] * sizeof(double)), "mg second guess");
		pinc_check(pinc_hip_fft_create(&S->fft, S->L[0].nd, S->L[0].T, g_pinc.stream), "mg second guess");
		pinc_check(pinc_hip_fft_set_symbol(S->fft, 1), "mg second guess");
	} else if (S->secondSpectral == 2) {
		long n = S->ps0 * S->nloc0;
		pinc_check(pinc_hip_malloc((void **)&S->rhoSave, n * sizeof(double)), "mg second guess");
		pinc_check(pinc_hip_malloc((void **)&S->dphi, n * sizeof(double)), "mg second guess");
		pinc_check(pinc_hip_fft_slab_create(&S->fftSlab, g.T, g.nloc, g_pinc.nranks, g_pinc.rank, g_pinc.stream),
		           "mg second guess");
		pinc_check(pinc_hip_fft_slab_set_symbol(S->fftSlab, 1), "mg second guess");
	}
	if (S->extrap && S->objects) {
		pinc_check(pinc_hip_malloc((void **)&S->phiA, S->N[0] * sizeof(double)), "mg extrapolation");
		pinc_check(pinc_hip_malloc((void **)&S->phiB, S->N[0] * sizeof(double)), "mg extrapolation");
		pinc_check(pinc_hip_malloc((void **)&S->dCorr, S->N[0] * sizeof(double)), "mg extrapolation");
	}
	S->rhoGrid = rho;
	S->phiGrid = phi;
	return S;
}

void mgFreeSolver(MultigridSolver *S) {
	if (!S) return;
	pinc_hip_graph_destroy(S->cycleGraph);
	pinc_hip_free(S->phiPrev);
	pinc_hip_free(S->phiA);
	pinc_hip_free(S->phiB);
	pinc_hip_free(S->dCorr);
	pinc_hip_free(S->rhoSave);
	pinc_hip_free(S->dphi);
	pinc_hip_fft_destroy(S->fft);
	pinc_hip_fft_slab_destroy(S->fftSlab);
	pinc_hip_fft_destroy(S->fftCoarse);
	pinc_hip_fft_slab_destroy(S->fftCoarseSlab);
	pinc_hip_free(S->phi1Ext);
	pinc_hip_host_free(S->hostNorm);
	pinc_hip_free(S->smallOut);
	pinc_hip_free(S->smallBasis);
	pinc_hip_host_free(S->hostSmall);
	if (S->normEvent) pinc_hip_event_destroy(S->normEvent);
	free(S->hist);
	for (int q = 0; q < S->nLevels; q++) {
		if (q > 0 || S->shard) {
			pinc_hip_free(S->rho[q]);
			pinc_hip_free(S->phi[q]);
		}
		pinc_hip_free(S->res[q]);
	}
	if (S->shard) {
		pinc_hip_free(S->rho1Slab);
		S->phiGrid->dev->ext = NULL; /* the grids outlive the solver (main.c:283-290) */
	}
	free(S);
}

long mgCycleCount(const MultigridSolver *S) { return S->cycles; }

void mgGuessNext(MultigridSolver *S, int role) {
	if (S && S->objects) S->role = role;
}

/* initial guess of a solve (multigrid:extrapolate); phi[0] holds the last
 * solution of this solver when a solve starts */
static void guess_begin(MultigridSolver *S, int role) {
	long n = S->N[0];
	double *phi = S->phi[0];
	if (role == PINC_MG_GUESS_SERIES) {
		/* 2 phi_n - phi_{n-1} once two solutions exist (the first solve
		 * starts from whatever phi held, the second from the first solution) */
		if (S->havePrev >= 2) pinc_check(pinc_hip_extrapolate(phi, S->phiPrev, n, g_pinc.stream), "mg extrapolation");
		else if (S->havePrev == 1) pinc_check(pinc_hip_d2d(S->phiPrev, phi, n * sizeof(double), g_pinc.stream), "mg extrapolation");
		if (S->havePrev < 2) S->havePrev++;
	} else if (role == PINC_MG_GUESS_FIRST && S->havePrev >= 2) {
		/* from the first solutions of the last two steps */
		pinc_check(pinc_hip_lincomb(phi, S->phiA, 2.0, S->phiB, -1.0, n, g_pinc.stream), "mg extrapolation");
	} else if (role == PINC_MG_GUESS_SECOND && S->secondSpectral == 1 && S->havePrev >= 1) {
		/* this step's first solution + the exact discrete response to the
		 * correction charge (rho now minus rho of the first solve) */
		pinc_check(pinc_hip_lincomb(S->rhoSave, S->rho[0], 1.0, S->rhoSave, -1.0, n, g_pinc.stream), "mg second guess");
		pinc_check(pinc_hip_fft_poisson(S->fft, S->rhoSave, S->dphi, g_pinc.stream), "mg second guess");
		pinc_check(pinc_hip_lincomb(phi, phi, 1.0, S->dphi, 1.0, n, g_pinc.stream), "mg second guess");
	} else if (role == PINC_MG_GUESS_SECOND && S->secondSpectral == 2 && S->havePrev >= 1) {
		/* the same on the sharded level 0: the owned planes of the correction
		 * charge through the slab-distributed transform; the halo planes of
		 * the guess are refreshed before the first smoothing chunk */
		long no = S->ps0 * S->nloc0, o = (long)S->hz * S->ps0;
		pinc_check(pinc_hip_lincomb(S->rhoSave, S->rho[0] + o, 1.0, S->rhoSave, -1.0, no, g_pinc.stream),
		           "mg second guess");
		pinc_slab_poisson(S->fftSlab, S->rhoSave, S->dphi, "mg second guess");
		pinc_check(pinc_hip_lincomb(phi + o, phi + o, 1.0, S->dphi, 1.0, no, g_pinc.stream), "mg second guess");
	} else if (role == PINC_MG_GUESS_SECOND && S->haveCorr) {
		/* this step's first solution + the last step's correction response */
		pinc_check(pinc_hip_lincomb(phi, phi, 1.0, S->dCorr, 1.0, n, g_pinc.stream), "mg extrapolation");
	}
}

static void guess_end(MultigridSolver *S, int role) {
	long n = S->N[0];
	if (role == PINC_MG_GUESS_FIRST) {
		double *t = S->phiB;
		S->phiB = S->phiA;
		S->phiA = t;
		pinc_check(pinc_hip_d2d(S->phiA, S->phi[0], n * sizeof(double), g_pinc.stream), "mg extrapolation");
		if (S->secondSpectral == 1)
			pinc_check(pinc_hip_d2d(S->rhoSave, S->rho[0], n * sizeof(double), g_pinc.stream), "mg second guess");
		else if (S->secondSpectral == 2)
			pinc_check(pinc_hip_d2d(S->rhoSave, S->rho[0] + (long)S->hz * S->ps0, S->ps0 * S->nloc0 * sizeof(double),
			                        g_pinc.stream),
			           "mg second guess");
		if (S->havePrev < 2) S->havePrev++;
	} else if (role == PINC_MG_GUESS_SECOND && S->havePrev >= 1) {
		pinc_check(pinc_hip_lincomb(S->dCorr, S->phi[0], 1.0, S->phiA, -1.0, n, g_pinc.stream), "mg extrapolation");
		S->haveCorr = 1;
	}
}

void mgSetLimit(MultigridSolver *S, long maxCycles, long histCap) {
	S->maxCycles = maxCycles > 0 ? maxCycles : 0;
	free(S->hist);
	S->hist = histCap > 0 ? calloc(histCap, sizeof(double)) : NULL;
	S->histCap = histCap > 0 ? histCap : 0;
	S->histN = 0;
}

int mgLevels(const MultigridSolver *S) { return S->nLevels; }

int mgShardHalo(const MultigridSolver *S) { return S->shard ? S->hz : 0; }

long mgHistory(const MultigridSolver *S, double *out, long cap) {
	long n = S->histN < S->histCap ? S->histN : S->histCap;
	if (out)
		for (long i = 0; i < n && i < cap; i++) out[i] = S->hist[i];
	return S->histN;
}

/* gNeutralizeGrid on a level of the global grid */
static void neutralize(double *a, long N) {
	pinc_check(pinc_hip_sum_div(a, N, (double)N, g_pinc.dScratch, PINC_SLOT(TMP_SLOT), g_pinc.stream), "mean");
	pinc_check(pinc_hip_sub_dev(a, N, PINC_SLOT(TMP_SLOT), g_pinc.stream), "neutralize");
}

/* sharded level 0: refresh the hz halo planes of an extended slab */
static void shard_halo(MultigridSolver *S, double *a) { pinc_ext_halo(a, S->ps0, S->nloc0, S->hz); }

/* gNeutralizeGrid of the sharded level 0: mean over the owned planes of
 * all ranks, subtracted from the whole extended slab */
static void neutralize_shard(MultigridSolver *S, double *a) {
	long ps = S->ps0;
	pinc_check(pinc_hip_sum(a + (long)S->hz * ps, ps * S->nloc0, g_pinc.dScratch, PINC_SLOT(TMP_SLOT), g_pinc.stream),
	           "mean");
	if (g_pinc.nranks > 1) pinc_comm_allreduce_sum(PINC_SLOT(TMP_SLOT), 1, "mg mean");
	pinc_check(pinc_hip_reduce(PINC_SLOT(TMP_SLOT), 1, (double)S->Ng0, PINC_SLOT(TMP_SLOT + 2), g_pinc.stream), "mean");
	pinc_check(pinc_hip_sub_dev(a, S->N[0], PINC_SLOT(TMP_SLOT + 2), g_pinc.stream), "neutralize");
}

static void neutralize_level(MultigridSolver *S, int q, double *a) {
	if (q == 0 && S->shard) neutralize_shard(S, a);
	else neutralize(a, S->N[q]);
}

/* phi[qf] += prolongated phi[qf + 1] */
static void prolong_into(MultigridSolver *S, int qf) {
	if (qf == 0 && S->dist1) {
		/* the owned planes only, from this rank's level-1 planes and one halo
		 * plane each side; the halo planes of level 0 come from the
		 * neighbours' owned planes at the refresh before the post-smoothing */
		pinc_lvl_t Lcx = S->L[1];
		Lcx.T[2] = S->nloc0 / 2 + 2;
		pinc_check(pinc_hip_prolong_add_own(S->phi[0], S->L[0], S->hz, S->nloc0, S->phi1Ext, Lcx, g_pinc.stream),
		           "prolong own planes");
		if (S->nPost <= 0) shard_halo(S, S->phi[0]);
	} else if (qf == 0 && S->shard)
		pinc_check(pinc_hip_prolong_add_slab(S->phi[0], S->L[0], S->z0, S->L[1].T[2] * 2, S->phi[1], S->L[1],
		                                     g_pinc.stream),
		           "prolong slab");
	else if (S->L[qf].nd == 3 && !((uintptr_t)S->phi[qf] & 15))
		pinc_check(pinc_hip_prolong_add3(S->phi[qf], S->phi[qf + 1], S->L[qf + 1], g_pinc.stream), "prolong");
	else pinc_check(pinc_hip_prolong_add(S->phi[qf], S->phi[qf + 1], S->L[qf], g_pinc.stream), "prolong");
}

/* residual of level q restricted into rho[q + 1] (times 4 in native mode) */
static void restrict_residual(MultigridSolver *S, int q) {
	if (q == 0 && S->shard) {
		/* the restriction reads fine planes h-1 .. h+nloc-1 */
		int h = S->hz;
		pinc_check(pinc_hip_residual_slab(S->res[0], S->phi[0], S->rho[0], S->L[0], h - 1, h + S->nloc0,
		                                  g_pinc.stream),
		           "residual slab");
		pinc_check(pinc_hip_restrict_slab(S->res[0], S->L[0], h, S->rho1Slab, S->L1s, S->restr3d, g_pinc.stream),
		           "restrict slab");
		long n1 = (long)S->L1s.T[0] * S->L1s.T[1] * S->L1s.T[2];
		if (S->dist1) return; /* level 1 stays in its slabs (vrec) */
		if (g_pinc.nranks > 1) pinc_comm_allgather(S->rho1Slab, S->rho[1], n1, "gather level 1");
		else pinc_check(pinc_hip_d2d(S->rho[1], S->rho1Slab, n1 * sizeof(double), g_pinc.stream), "level 1");
		return;
	}
	if (S->L[q].nd == 3) {
		/* residual and restriction in one pass (the fine residual is never
		 * stored); the native x4 folded in */
		pinc_check(pinc_hip_resid_restrict(S->phi[q], S->rho[q], S->rho[q + 1], S->L[q + 1], S->restr3d,
		                                   S->native ? 4.0 : 1.0, g_pinc.stream),
		           "residual restrict");
		return;
	}
	pinc_check(pinc_hip_residual(S->res[q], S->phi[q], S->rho[q], S->L[q], g_pinc.stream), "residual");
	pinc_check(pinc_hip_restrict(S->res[q], S->rho[q + 1], S->L[q + 1], S->restr3d, g_pinc.stream), "restrict");
	if (S->native) pinc_check(pinc_hip_scale(S->rho[q + 1], S->N[q + 1], 4.0, g_pinc.stream), "native scale");
}

/* nIter red-black iterations, each colour followed by a neutralisation:
 * the mean of pass k is formed from that pass's partial sums and applied
 * lazily by pass k+1 (k_mg.hip), then materialised once at the end. */
/* native mode: red-black iterations without the per-colour neutralisation;
 * full sweeps in one pass where the level tiles (pinc_hip_gs_sweep, ping-pong
 * through res[q], which is free while smoothing), an odd last one in place */
static void smooth_native(MultigridSolver *S, int q, int nIter, int nd3) {
	const pinc_lvl_t L = S->L[q];
	/* the z-marching fused sweep pays off on large levels only (measured at
	 * 256^3: 128^3 and below are as fast, launch-latency bound, as two
	 * passes; rechecked with the 32x8 two-ahead sweep) */
	int fused = nd3 && L.nd == 3 && L.T[0] % 16 == 0 && L.T[1] % 16 == 0 && L.T[2] % 16 == 0 &&
	            (S->N[q] >= S->fusedMin || (q == 0 && S->shard && S->N[q] >= S->fusedMin / 4));
	int k = 0;
	/* two iterations per launch (pinc_hip_gs_sweep2x) in pairs, so that the
	 * ping-pong ends in phi */
	/* (its x-pair fetches need 16-B aligned arrays: otherwise the single
	 * sweeps, as the residual norm and the restriction fall back to their
	 * scalar kernels -- every x-pair kernel falls back, none fails) */
	int fused2 = fused && L.T[0] % 32 == 0 && L.T[1] % 8 == 0 &&
	             !(((uintptr_t)S->phi[q] | (uintptr_t)S->res[q] | (uintptr_t)S->rho[q]) & 15);
	if (q == 0 && S->preDone) {
		/* the first double sweep ran while the host read the last cycle's
		 * norm (mgSolve), and its ping-pong swap is applied */
		if (!(fused2 && !S->shard && nIter >= 2)) msg(ERROR, "mg: a speculative sweep the smoothing cannot use");
		S->preDone = 0;
		k = 2;
	}
	if (fused2 && !(q == 0 && S->shard)) {
		/* one launch per two iterations, phi[q] -> res[q], then the pointers
		 * swap (round 4: a smoothing of 10 is five double sweeps instead of
		 * four and a pair of single ones; the V-cycle's other kernels take
		 * whichever buffer holds the iterate, pp_restore puts it back) */
		for (; k + 2 <= nIter; k += 2) {
			int slot = q == 0 && (k & 2) == 0 ? pinc_probe_begin(PINC_PROBE_GS) : -1;
			if (q == 0 && (k & 2)) pinc_probe_count(PINC_PROBE_GS);
			pinc_check(pinc_hip_gs_sweep2x(S->phi[q], S->res[q], S->rho[q], L, g_pinc.stream), "gs sweep2x");
			pinc_probe_end(PINC_PROBE_GS, slot, 24.0 * S->N[q]);
			double *t = S->phi[q];
			S->phi[q] = S->res[q];
			S->res[q] = t;
			S->swapped[q] ^= 1;
		}
	}
	if (fused2 && q == 0 && S->shard) {
		for (; k + 4 <= nIter; k += 4) {
			int slot = q == 0 ? pinc_probe_begin(PINC_PROBE_GS) : -1;
			pinc_check(pinc_hip_gs_sweep2x(S->phi[q], S->res[q], S->rho[q], L, g_pinc.stream), "gs sweep2x");
			/* two full iterations: phi R + W, rho R (24 B per point) once */
			pinc_probe_end(PINC_PROBE_GS, slot, 24.0 * S->N[q]);
			pinc_probe_count(PINC_PROBE_GS);
			pinc_check(pinc_hip_gs_sweep2x(S->res[q], S->phi[q], S->rho[q], L, g_pinc.stream), "gs sweep2x");
		}
	}
	if (fused) {
		for (; k + 2 <= nIter; k += 2) {
			int slot = q == 0 && !fused2 ? pinc_probe_begin(PINC_PROBE_GS) : -1;
			pinc_check(pinc_hip_gs_sweep(S->phi[q], S->res[q], S->rho[q], L, g_pinc.stream), "gs sweep");
			/* one full iteration: phi R + W, rho R (24 B per point) */
			pinc_probe_end(PINC_PROBE_GS, slot, 24.0 * S->N[q]);
			if (q == 0 && !fused2) pinc_probe_count(PINC_PROBE_GS);
			pinc_check(pinc_hip_gs_sweep(S->res[q], S->phi[q], S->rho[q], L, g_pinc.stream), "gs sweep");
		}
	}
	for (; k < nIter; k++) {
		for (int pass = 0; pass < 2; pass++) {
			int nb = 0;
			pinc_check(pinc_hip_gs_pass(S->phi[q], S->rho[q], L, pass, nd3, NULL, NULL, &nb, g_pinc.stream),
			           "gs pass");
		}
	}
}

/* level 0's pre-smoothing opens with one pinc_hip_gs_sweep2x phi -> res
 * (smooth_native's fused2 branch): the sweep mgSolve may queue ahead */
static int first_sweep_is_double(const MultigridSolver *S) {
	const pinc_lvl_t L = S->L[0];
	if (!S->native || S->shard || S->nPre < 2 || !S->pre3d) return 0;
	int fused = L.nd == 3 && L.T[0] % 16 == 0 && L.T[1] % 16 == 0 && L.T[2] % 16 == 0 && S->N[0] >= S->fusedMin;
	return fused && L.T[0] % 32 == 0 && L.T[1] % 8 == 0 &&
	       !(((uintptr_t)S->phi[0] | (uintptr_t)S->res[0] | (uintptr_t)S->rho[0]) & 15);
}

/* the iterate back into phi[q]'s own buffer after a swapped smoothing */
static void pp_restore(MultigridSolver *S, int q) {
	if (!S->swapped[q]) return;
	pinc_check(pinc_hip_d2d(S->res[q], S->phi[q], S->N[q] * sizeof(double), g_pinc.stream), "mg ping-pong");
	double *t = S->phi[q];
	S->phi[q] = S->res[q];
	S->res[q] = t;
	S->swapped[q] = 0;
}

static void smooth(MultigridSolver *S, int q, int nIter, int nd3) {
	if (nIter <= 0) return;
	if (q == 0 && S->shard) {
		for (int k = 0; k < nIter; k += S->chunk) {
			shard_halo(S, S->phi[0]);
			smooth_native(S, 0, nIter - k < S->chunk ? nIter - k : S->chunk, nd3);
		}
		return;
	}
	if (S->native) {
		smooth_native(S, q, nIter, nd3);
		return;
	}
	int nPass = 2 * nIter;
	for (int k = 0; k < nPass; k++) {
		const double *muPrev = k ? PINC_SLOT(MU_SLOT + ((k - 1) & 1)) : NULL;
		int nb = 0;
		/* algorithmic bytes of one colour pass: half of a
		 * red+black iteration's 24 B per point (phi R+W, rho R) */
		int slot = q == 0 ? pinc_probe_begin(PINC_PROBE_GS) : -1;
		pinc_check(pinc_hip_gs_pass(S->phi[q], S->rho[q], S->L[q], k & 1, nd3, muPrev, g_pinc.dScratch, &nb,
		                            g_pinc.stream),
		           "gs pass");
		pinc_probe_end(PINC_PROBE_GS, slot, 12.0 * S->N[q]);
		pinc_check(pinc_hip_reduce(g_pinc.dScratch, nb, (double)S->N[q], PINC_SLOT(MU_SLOT + (k & 1)), g_pinc.stream),
		           "gs mean");
	}
	pinc_check(pinc_hip_gs_materialize(S->phi[q], S->L[q], 1, PINC_SLOT(MU_SLOT), PINC_SLOT(MU_SLOT + 1),
	                                   g_pinc.stream),
	           "gs materialize");
}

/* native mode: first level from which the rest of the V-cycle fits the
 * single-workgroup LDS kernel (pinc_hip_mg_coarse), or -1.  Its smoother is
 * one form for every phase (all three 3-D, or all three N-D).  (A variant
 * that also ran level 0 of small grids in that one workgroup, from L2, was
 * slower at C2's 128^2: 3.7 ms per solve against 2.2 ms.) */
static int coarse_start(const MultigridSolver *S) {
	if (!S->native) return -1;
	int all3 = S->pre3d && S->post3d && S->coarse3d, none3 = !S->pre3d && !S->post3d && !S->coarse3d;
	if (!all3 && !none3) return -1;
	for (int q = 1; q < S->nLevels; q++) {
		if (S->N[q] > 4096) continue;
		long tot = 0;
		for (int k = q; k < S->nLevels; k++) tot += 3 * S->N[k];
		if (tot <= 5500 * 3 && S->nLevels - q <= 12) return q;
	}
	return -1;
}

static void vrec(MultigridSolver *S, int q) {
	int bottom = S->nLevels - 1;
	if (S->dist1 && q == 1) {
		/* two-grid cycle, level 1 decomposed: this rank's restricted
		 * residual planes through the slab-distributed transform with the
		 * 7-point symbol (DC dropped), then one level-1 halo plane from each
		 * neighbour for the prolongation */
		const long ps1 = (long)S->L[1].T[0] * S->L[1].T[1];
		const int n1 = S->nloc0 / 2;
		pinc_slab_poisson(S->fftCoarseSlab, S->rho1Slab, S->phi1Ext + ps1, "mg spectral coarse (slabs)");
		pinc_ext_halo(S->phi1Ext, ps1, n1, 1);
		prolong_into(S, 0);
		return;
	}
	if (S->fftCoarse && q == 1) {
		/* two-grid cycle with an exact coarse solve: the level-1 correction
		 * equation -L phi1 = rho1 (rho1 the restricted residual, times 4)
		 * solved by FFT with the 7-point symbol; DC dropped (neutral) */
		pinc_check(pinc_hip_fft_poisson(S->fftCoarse, S->rho[1], S->phi[1], g_pinc.stream), "mg spectral coarse");
		prolong_into(S, 0);
		return;
	}
	int qc = coarse_start(S);
	if (qc > 0 && q == qc) {
		pinc_check(pinc_hip_mg_coarse(S->rho[q], S->phi[q], S->nLevels - q, &S->L[q], S->nPre, S->nPost, S->nCoarse,
		                              S->restr3d, S->pre3d, g_pinc.stream),
		           "mg coarse");
		prolong_into(S, q - 1);
		return;
	}
	/* native mode: correction scheme, each coarse visit solves for the
	 * correction from zero (the reference warm-starts coarse phi) */
	if (S->native && q > 0) pinc_check(pinc_hip_zero(S->phi[q], S->N[q], g_pinc.stream), "native zero");
	if (q == bottom) {
		neutralize(S->rho[q], S->N[q]);
		smooth(S, q, S->nCoarse, S->coarse3d);
		neutralize(S->phi[q], S->N[q]);
		pp_restore(S, q);
		prolong_into(S, q - 1);
		return;
	}
	/* native mode: level 0's rho and phi are neutralised once per solve
	 * (mgSolve), not per cycle -- rho does not change during the solve, and
	 * the V-cycle commutes with adding a constant to phi (the residual,
	 * hence the correction, does not see it; the smoother carries it) -- and
	 * no level's phi between the prolongation and the post-smoothing, for the
	 * same reason (round 4; the oracle's native solve mirrors this) */
	if (!(S->native && q == 0)) neutralize_level(S, q, S->rho[q]);
	smooth(S, q, S->nPre, S->pre3d);
	restrict_residual(S, q);
	vrec(S, q + 1);
	if (!S->native) neutralize_level(S, q, S->phi[q]);
	smooth(S, q, S->nPost, S->post3d);
	if (!(S->native && q == 0)) neutralize_level(S, q, S->phi[q]);
	pp_restore(S, q);
	if (q > 0) prolong_into(S, q - 1);
}

void mgSolve(MultigridSolver *S, Grid *rho, Grid *phi, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	(void)phi;
	pinc_phase_begin(4);
	if (S->shard) {
		/* this rank's rho into the extended slab, halo from the neighbours */
		long ps = S->ps0;
		pinc_check(pinc_hip_d2d(S->rho[0] + (long)S->hz * ps, rho->dev->d + ps, ps * S->nloc0 * sizeof(double),
		                        g_pinc.stream),
		           "shard rho");
		shard_halo(S, S->rho[0]);
	} else if (g_pinc.nranks > 1) {
		long ps = rho->dev->planeSize;
		pinc_comm_allgather(rho->dev->d + ps, rho->dev->global, ps * rho->dev->geom.nloc, "gather rho");
	}
	const int role = S->extrap ? S->role : PINC_MG_GUESS_WARM;
	guess_begin(S, role);
	if (S->nLevels > 1) {
		/* the reference loops until converged (multigrid.c:1698); PINC_MG_MAX_CYCLES
		 * caps a solve for diagnostics (stops with a warning) */
		const long maxCycles = 1000000;
		const char *capEnv = getenv("PINC_MG_MAX_CYCLES");
		long cap = S->maxCycles ? S->maxCycles : (capEnv ? atol(capEnv) : 0);
		double barRes = 2.;
		long c = 0;
		S->histN = 0;
		if (S->native) neutralize_level(S, 0, S->rho[0]);
		if (S->small) {
			c = small_solve(S, cap, &barRes);
			if (!(S->maxCycles && !isfinite(barRes)) && (!isfinite(barRes) || (c > maxCycles && barRes > 1.E-10)))
				msg(ERROR, "multigrid did not converge (residual %g)", barRes);
			if (!isfinite(barRes))
				fprintf(stderr, "[pinc] rank %d solve stopped: residual %g after %ld cycles\n", g_pinc.rank, barRes, c);
			else if (cap > 0 && c >= cap && barRes > 1.E-10)
				fprintf(stderr, "[pinc] rank %d solve stopped at the PINC_MG_MAX_CYCLES cap (%ld), residual %.3e\n",
				        g_pinc.rank, c, barRes);
			barRes = 0; /* the loop below is the multi-launch form */
		}
		while (barRes > 1.E-10) {
			if (S->useGraph) {
				/* the V-cycle is a fixed launch sequence on fixed buffers:
				 * captured once, then replayed (no per-kernel dispatch) */
				if (!S->cycleGraph) {
					g_pinc.capturing = 1;
					pinc_check(pinc_hip_capture_begin(g_pinc.stream), "capture V-cycle");
					vrec(S, 0);
					pinc_check(pinc_hip_capture_end(g_pinc.stream, &S->cycleGraph), "capture V-cycle");
					g_pinc.capturing = 0;
				}
				int gslot = pinc_probe_begin(PINC_PROBE_CYCLE);
				pinc_check(pinc_hip_graph_launch(S->cycleGraph, g_pinc.stream), "V-cycle graph");
				pinc_probe_end(PINC_PROBE_CYCLE, gslot, 0.0);
			} else {
				vrec(S, 0);
			}
			S->cycles++;
			int nb = 0;
			int slot = pinc_probe_begin(PINC_PROBE_RESIDUAL);
			if (S->shard) {
				/* owned planes, summed over the ranks */
				pinc_check(pinc_hip_residual_sumsq_slab(S->phi[0], S->rho[0], S->L[0], S->hz, S->hz + S->nloc0,
				                                        g_pinc.dScratch, &nb, g_pinc.stream),
				           "residual norm");
				pinc_probe_end(PINC_PROBE_RESIDUAL, slot, 16.0 * S->ps0 * S->nloc0);
				pinc_check(pinc_hip_reduce(g_pinc.dScratch, nb, 1.0, PINC_SLOT(TMP_SLOT + 1), g_pinc.stream), "norm");
				if (g_pinc.nranks > 1) pinc_comm_allreduce_sum(PINC_SLOT(TMP_SLOT + 1), 1, "norm");
			} else {
				pinc_check(pinc_hip_residual_sumsq(S->phi[0], S->rho[0], S->L[0], g_pinc.dScratch, &nb, g_pinc.stream),
				           "residual norm");
				pinc_probe_end(PINC_PROBE_RESIDUAL, slot, 16.0 * S->N[0]);
				pinc_check(pinc_hip_reduce(g_pinc.dScratch, nb, 1.0, PINC_SLOT(TMP_SLOT + 1), g_pinc.stream), "norm");
			}
			double sum = 0;
			int spec = 0;
			if (S->speculate) {
				/* the norm to pinned memory; while the host waits for it, the
				 * next cycle's first double sweep (phi -> res: phi untouched)
				 * runs if the last solve of this role needed another cycle */
				pinc_check(pinc_hip_d2h_async(S->hostNorm, PINC_SLOT(TMP_SLOT + 1), sizeof(double), g_pinc.stream),
				           "norm");
				pinc_check(pinc_hip_event_record(S->normEvent, g_pinc.stream), "norm");
				spec = first_sweep_is_double(S) && c + 1 < S->lastCycles[role & 3] && !S->swapped[0];
				if (spec) {
					int gslot = pinc_probe_begin(PINC_PROBE_GS);
					pinc_check(pinc_hip_gs_sweep2x(S->phi[0], S->res[0], S->rho[0], S->L[0], g_pinc.stream),
					           "gs sweep2x (ahead)");
					pinc_probe_end(PINC_PROBE_GS, gslot, 24.0 * S->N[0]);
				}
				pinc_check(pinc_hip_event_sync(S->normEvent), "norm");
				sum = *S->hostNorm;
			} else {
				pinc_check(pinc_hip_d2h(S->hostNorm, PINC_SLOT(TMP_SLOT + 1), sizeof(double), g_pinc.stream), "norm");
				sum = *S->hostNorm;
			}
			barRes = sqrt(sum / S->Ng0);
			if (S->histN < S->histCap) S->hist[S->histN] = barRes;
			S->histN++;
			if (S->maxCycles && !isfinite(barRes)) {
				/* diagnostic run (mgSetLimit): keep the history, stop */
				fprintf(stderr, "[pinc] rank %d solve stopped: residual %g after %ld cycles\n", g_pinc.rank, barRes, c + 1);
				break;
			}
			if (++c > maxCycles || isnan(barRes)) msg(ERROR, "multigrid did not converge (residual %g)", barRes);
			if (g_pinc.verbose && (c % g_pinc.verbose == 0)) {
				fprintf(stderr, "[pinc] rank %d solve cycle %ld residual %.3e\n", g_pinc.rank, c, barRes);
				fflush(stderr);
			}
			if (cap > 0 && c >= cap) {
				fprintf(stderr, "[pinc] rank %d solve stopped at the PINC_MG_MAX_CYCLES cap (%ld), residual %.3e\n",
				        g_pinc.rank, c, barRes);
				break;
			}
			if (spec && barRes > 1.E-10) {
				/* another cycle: its first double sweep is done (the
				 * smoothing's ping-pong swap now) */
				double *t = S->phi[0];
				S->phi[0] = S->res[0];
				S->res[0] = t;
				S->swapped[0] ^= 1;
				S->preDone = 1;
			}
		}
		S->preDone = 0;
		S->lastCycles[role & 3] = c;
		if (S->native) neutralize_level(S, 0, S->phi[0]);
	} else {
		for (int c = 0; c < S->mgCycles; c++) {
			neutralize(S->rho[0], S->N[0]);
			smooth(S, 0, S->nCoarse, S->coarse3d);
			pp_restore(S, 0);
		}
	}
	guess_end(S, role);
	if (S->objects) S->role = PINC_MG_GUESS_WARM; /* mgGuessNext holds for one solve */
	phi->dev->ghostsValid = 0;
	if (S->shard) {
		/* the slab with its ghost planes (exact: within hz - 2 chunk of the
		 * owned planes); E reads the extended slab directly (gFinDiff1st) */
		long ps = S->ps0;
		pinc_check(pinc_hip_d2d(phi->dev->d, S->phi[0] + (long)(S->hz - 1) * ps, ps * (S->nloc0 + 2) * sizeof(double),
		                        g_pinc.stream),
		           "shard phi");
		phi->dev->ghostsValid = 1;
		phi->dev->extStale = 0;
	}
	pinc_phase_end(4);
}
