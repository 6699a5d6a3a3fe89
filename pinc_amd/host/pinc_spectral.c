/*
 * pinc_spectral.c -- spectral Poisson solver of the MI355X PINC hot path
 * (host C), the solver triple of src/spectral.c:
 *
 *   sSolver / sSolver_set   spectral.c:62-89 (solver interface + checks)
 *   sAlloc                  spectral.c:14-52: plans for the true grid
 *   sSolve                  spectral.c:92-115: r2c, DC := 0, multiply by
 *                           (N/2 pi n)^2/N, c2r (rocFFT, k_spectral.hip)
 *   sFree                   spectral.c:54-60
 *
 * The reference is 1-D only (sSolver_set rejects nDims != 1 and any
 * decomposition).  This build runs the same operator in 1, 2 or 3
 * dimensions: the factor becomes 1/|k|^2/N over the whole periodic domain.
 * With several ranks in 3-D (Ty divisible by the rank count, no objects,
 * spectral:distributed not 0) the solve is slab-distributed (SURVEY.md
 * 8(f)4; k_spectral.hip): 2-D transforms of each rank's planes, an
 * all-to-all transpose to ky blocks, transforms along z, and back, so rho
 * is never gathered; phi lands in each rank's slab and E is taken from the
 * slab (its ghost planes exchanged).  Otherwise the rho slabs are
 * all-gathered (RCCL) and every rank transforms the global grid, as the
 * replicated multigrid solve does; each rank's phi slab is then a view of
 * the global phi, copied into the slab by the TOHALO after every solve.
 */
#define _GNU_SOURCE
#include "pinc_internal.h"

static void all_to_all(char *src, char *dst, long blockBytes, const char *what);

struct SpectralSolver {
	pinc_fft_t *fft;
	pinc_fft_slab_t *slab;  /* slab-distributed plan (several ranks, 3-D) */
	long N;
	long solves;
};

void sSolver(void (**solve)(), void *(**solverAlloc)(), void (**solverFree)()) {
	*solve = (void (*)())sSolve;
	*solverAlloc = (void *(*)())sAlloc;
	*solverFree = (void (*)())sFree;
}

funPtr sSolver_set(dictionary *ini) {
	int nd = iniGetInt(ini, "grid:nDims");
	if (nd < 1 || nd > 3) msg(ERROR, "sSolver supports grid:nDims=1..3");
	int *ts = iniGetIntArr(ini, "grid:trueSize", nd);
	int *ns = iniGetIntArr(ini, "grid:nSubdomains", nd);
	if (ts[0] * ns[0] % 2) msg(ERROR, "sSolver needs an even global grid:trueSize along x");
	free(ts);
	free(ns);
	return (funPtr)sSolver;
}

SpectralSolver *sAlloc(const dictionary *ini, Grid *rho, Grid *phi) {
	(void)ini;
	SpectralSolver *S = calloc(1, sizeof(*S));
	pinc_geom_t g = rho->dev->geom;
	S->N = 1;
	for (int d = 0; d < g.nd; d++) S->N *= g.T[d];
	long ps = rho->dev->planeSize;
	int objects = iniHas(ini, "objects:sphere") || iniHas(ini, "objects:file");
	int dist = !iniHas(ini, "spectral:distributed") || iniGetInt(ini, "spectral:distributed");
	if (g_pinc.nranks > 1 && g.nd == 3 && g.T[1] % g_pinc.nranks == 0 && !objects && dist) {
		pinc_check(pinc_hip_fft_slab_create(&S->slab, g.T, g.nloc, g_pinc.nranks, g_pinc.rank, g_pinc.stream),
		           "rocFFT slab plans");
		/* E from the slab: its ghost planes come from the neighbours */
		phi->dev->ext = phi->dev->d;
		phi->dev->extOff = 1;
		phi->dev->extPlanes = g.nloc + 2;
		return S;
	}
	pinc_check(pinc_hip_fft_create(&S->fft, g.nd, g.T, g_pinc.stream), "rocFFT plans");
	if (g_pinc.nranks == 1) {
		rho->dev->global = rho->dev->d + ps;
		phi->dev->global = phi->dev->d + ps;
		phi->dev->globalIsTruth = 1;
	} else if (!rho->dev->global) {
		pinc_check(pinc_hip_malloc((void **)&rho->dev->global, S->N * sizeof(double)), "global rho");
		pinc_check(pinc_hip_malloc((void **)&phi->dev->global, S->N * sizeof(double)), "global phi");
		pinc_check(pinc_hip_memset(phi->dev->global, 0, S->N * sizeof(double), g_pinc.stream), "global phi");
		rho->dev->ownsGlobal = phi->dev->ownsGlobal = 1;
		phi->dev->globalIsTruth = 1;
	}
	return S;
}

/* phi slab = the plan's Poisson operator on the rho slab (nloc planes each,
 * no ghosts), slab-distributed over the ranks */
void pinc_slab_poisson(pinc_fft_slab_t *plan, const double *rhoSlab, double *phiSlab, const char *what) {
	void *sBuf = NULL, *bBuf = NULL;
	long blk = 0;
	pinc_check(pinc_hip_fft_slab_buffers(plan, &sBuf, &bBuf, &blk), what);
	pinc_check(pinc_hip_fft_slab_forward(plan, rhoSlab, g_pinc.stream), what);
	all_to_all(sBuf, bBuf, blk, what);
	pinc_check(pinc_hip_fft_slab_kspace(plan, g_pinc.stream), what);
	all_to_all(bBuf, sBuf, blk, what);
	pinc_check(pinc_hip_fft_slab_backward(plan, phiSlab, g_pinc.stream), what);
}

void sFree(SpectralSolver *S) {
	if (!S) return;
	pinc_hip_fft_destroy(S->fft);
	pinc_hip_fft_slab_destroy(S->slab);
	free(S);
}

/* all-to-all of P blocks: block q of src goes to rank q, block p of dst
 * comes from rank p (this rank's own block by a device copy) */
static void all_to_all(char *src, char *dst, long blockBytes, const char *what) {
	int P = g_pinc.nranks, r = g_pinc.rank, n = P - 1;
	int *sp = malloc(n * sizeof(int)), *rp = malloc(n * sizeof(int));
	void **sb = malloc(n * sizeof(void *)), **rb = malloc(n * sizeof(void *));
	long *nb = malloc(n * sizeof(long));
	for (int i = 1; i < P; i++) {
		sp[i - 1] = (r + i) % P;
		rp[i - 1] = (r - i + P) % P;
		sb[i - 1] = src + (long)sp[i - 1] * blockBytes;
		rb[i - 1] = dst + (long)rp[i - 1] * blockBytes;
		nb[i - 1] = blockBytes;
	}
	pinc_check(pinc_hip_d2d(dst + (long)r * blockBytes, src + (long)r * blockBytes, blockBytes, g_pinc.stream), what);
	if (n > 0) pinc_comm_exchange(n, sp, sb, nb, rp, rb, nb, what);
	free(sp);
	free(rp);
	free(sb);
	free(rb);
	free(nb);
}

void sSolve(SpectralSolver *S, Grid *rho, Grid *phi, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	pinc_phase_begin(4);
	if (S->slab) {
		long ps = rho->dev->planeSize;
		int slot = pinc_probe_begin(PINC_PROBE_SPECTRAL);
		pinc_slab_poisson(S->slab, rho->dev->d + ps, phi->dev->d + ps, "spectral transpose");
		pinc_probe_end(PINC_PROBE_SPECTRAL, slot, 48.0 * S->N / g_pinc.nranks);
		S->solves++;
		phi->dev->ghostsValid = 0;
		phi->dev->extStale = 1;  /* the slab's ghost planes: exchanged before E */
		pinc_phase_end(4);
		return;
	}
	if (g_pinc.nranks > 1) {
		long ps = rho->dev->planeSize;
		pinc_comm_allgather(rho->dev->d + ps, rho->dev->global, ps * rho->dev->geom.nloc, "gather rho");
	}
	int slot = pinc_probe_begin(PINC_PROBE_SPECTRAL);
	pinc_check(pinc_hip_fft_poisson(S->fft, rho->dev->global, phi->dev->global, g_pinc.stream), "spectral solve");
	/* algorithmic bytes, one HBM pass per stage:
	 * r2c rho R 8 + spectrum W 8, scale R+W 16, c2r R 8 + phi W 8 per point */
	pinc_probe_end(PINC_PROBE_SPECTRAL, slot, 48.0 * S->N);
	S->solves++;
	phi->dev->ghostsValid = 0;
	pinc_phase_end(4);
}

long sSolveCount(const SpectralSolver *S) { return S->solves; }

int sSolveDistributed(const SpectralSolver *S) { return S->slab != NULL; }
