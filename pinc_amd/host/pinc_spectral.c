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
 * With several ranks the rho slabs are all-gathered first (RCCL) and every
 * rank transforms the global grid, as the multigrid solver does here
 * (DESIGN.md "Poisson solve"); each rank's phi slab is then a view of the
 * global phi, copied into the slab by the TOHALO that follows every solve.
 */
#define _GNU_SOURCE
#include "pinc_internal.h"

struct SpectralSolver {
	pinc_fft_t *fft;
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
	pinc_check(pinc_hip_fft_create(&S->fft, g.nd, g.T, g_pinc.stream), "rocFFT plans");
	long ps = rho->dev->planeSize;
	if (g_pinc.nranks == 1) {
		rho->dev->global = rho->dev->d + ps;
		phi->dev->global = phi->dev->d + ps;
	} else if (!rho->dev->global) {
		pinc_check(pinc_hip_malloc((void **)&rho->dev->global, S->N * sizeof(double)), "global rho");
		pinc_check(pinc_hip_malloc((void **)&phi->dev->global, S->N * sizeof(double)), "global phi");
		pinc_check(pinc_hip_memset(phi->dev->global, 0, S->N * sizeof(double), g_pinc.stream), "global phi");
		rho->dev->ownsGlobal = phi->dev->ownsGlobal = 1;
	}
	return S;
}

void sFree(SpectralSolver *S) {
	if (!S) return;
	pinc_hip_fft_destroy(S->fft);
	free(S);
}

void sSolve(SpectralSolver *S, Grid *rho, Grid *phi, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	pinc_phase_begin(4);
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
