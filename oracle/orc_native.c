/*
 * orc_native.c -- TEST INFRASTRUCTURE (oracle).  The "native mode" multigrid
 * solve of the MI355X build (multigrid:native = 1; pinc_amd/host/pinc_mg.c,
 * DESIGN.md section 6), restated on the CPU so that the device's native
 * solver is checked cycle by cycle and the CPU baseline runs the same
 * algorithm as the GPU.  It is NOT in the reference: the reference's solver
 * (orc_mg.c, multigrid.c:1496-1556) omits the coarse h^2 factor and
 * warm-starts the coarse levels.  Native mode keeps the reference's
 * operators and their expression order --
 *   red-black Gauss-Seidel   mgGS3D / mgGSND   multigrid.c:553-767
 *   residual                 mgResidual        multigrid.c:1385-1403
 *   half-weight restriction  mgHalfRestrict*   multigrid.c:844-1022
 *   bilinear prolongation    mgBilinProl*      multigrid.c:1024-1238
 *   neutralisation           gNeutralizeGrid   grid.c:730-779
 *   stop at RMS residual <= 1e-10              multigrid.c:1688-1724
 * -- and changes the cycle: the restricted residual is scaled by 4 (the
 * coarse h^2), every coarse visit starts from zero (correction scheme), no
 * neutralisation after each colour (once per level visit instead; level 0's
 * rho and phi once per solve; none between prolongation and post-smoothing), and the
 * hierarchy continues down to 2 points per dimension.
 *
 * The solve runs on the global periodic grid (no ghosts, x fastest),
 * gathered from and scattered to the emulated ranks' true nodes, as the
 * device runs it.  Stencil loops are OpenMP-parallel (order-independent:
 * bit-identical for any thread count); sums are serial.
 */
#include "orc.h"
#include <math.h>

#define ON_MAX_LEVELS 12  /* PINC_MAX_LEVELS, include/pinc_hip.h */

typedef struct {
	int nd, T[3];
	long s[3], N;
} NLv;

struct ONative {
	int nLevels;
	NLv L[ON_MAX_LEVELS];
	double *rho[ON_MAX_LEVELS], *phi[ON_MAX_LEVELS], *res[ON_MAX_LEVELS];
	int nd3;        /* 3-D GS / restriction forms (gaussSeidelRB, halfWeight) */
	/* multigrid:extrapolate (pinc_mg.c guess_begin / guess_end): without
	 * objects 2 phi_n - phi_{n-1} once two solutions exist (prev holds
	 * phi_{n-1}, nSeen counts solves); with objects the first solve of a
	 * step from the first solutions of the last two steps (A, B), the
	 * second as the first plus the last step's correction response (D) */
	int extrap, nSeen, objects, role, haveCorr;
	double *prev, *A, *B, *D;
	/* objects:secondGuess = spectral: rho of the first solve, the exact
	 * discrete response to the correction charge (orc_discrete_poisson) */
	int secondSpectral;
	double *rhoSave, *dphi;
	int spectralCoarse;  /* multigrid:spectralCoarse */
};

static NLv mklv(int nd, const int *T){
	NLv l; l.nd = nd; l.N = 1;
	for(int d = 0; d < 3; d++){ l.T[d] = d < nd ? T[d] : 1; l.N *= l.T[d]; }
	l.s[0] = 1; l.s[1] = l.T[0]; l.s[2] = (long)l.T[0]*l.T[1];
	return l;
}

/* level count of the device solver: the ini's mgLevels, then halving on
 * while every dimension stays even with at least 2 points (pinc_mg.c) */
ONative *on_alloc(int nd, const int *Tg, int nLevelsIni, int nd3){
	ONative *S = calloc(1, sizeof(*S));
	int L = nLevelsIni;
	for(;;){
		int ok = L < ON_MAX_LEVELS;
		for(int d = 0; d < nd && ok; d++){ int t = Tg[d] >> (L-1); ok = (t % 2 == 0) && t/2 >= 2; }
		if(!ok) break;
		L++;
	}
	S->nLevels = L;
	S->nd3 = nd3;
	for(int q = 0; q < L; q++){
		int T[3];
		for(int d = 0; d < 3; d++) T[d] = d < nd ? Tg[d] >> q : 1;
		S->L[q] = mklv(nd, T);
		S->rho[q] = calloc(S->L[q].N, sizeof(double));
		S->phi[q] = calloc(S->L[q].N, sizeof(double));
		S->res[q] = calloc(S->L[q].N, sizeof(double));
	}
	return S;
}

void on_set_extrapolate(ONative *S, int on, int objects){
	long N = S->L[0].N;
	S->extrap = on;
	S->objects = objects;
	S->role = objects ? ON_GUESS_WARM : ON_GUESS_SERIES;
	if(on && !objects && !S->prev) S->prev = calloc(N, sizeof(double));
	if(on && objects && !S->A){
		S->A = calloc(N, sizeof(double));
		S->B = calloc(N, sizeof(double));
		S->D = calloc(N, sizeof(double));
	}
}

void on_guess_next(ONative *S, int role){ if(S->objects) S->role = role; }

void on_set_spectral_coarse(ONative *S, int on){ S->spectralCoarse = on && S->nLevels >= 2; }

void on_set_second_spectral(ONative *S, int on){
	S->secondSpectral = on && S->extrap && S->objects;
	if(S->secondSpectral && !S->rhoSave){
		S->rhoSave = calloc(S->L[0].N, sizeof(double));
		S->dphi = calloc(S->L[0].N, sizeof(double));
	}
}

void on_free(ONative *S){
	if(!S) return;
	free(S->prev); free(S->A); free(S->B); free(S->D); free(S->rhoSave); free(S->dphi);
	for(int q = 0; q < S->nLevels; q++){ free(S->rho[q]); free(S->phi[q]); free(S->res[q]); }
	free(S);
}

int on_levels(const ONative *S){ return S->nLevels; }

static inline void coords(const NLv *L, long g, int *c){
	c[0] = (int)(g % L->T[0]);
	long r = g / L->T[0];
	c[1] = (int)(r % L->T[1]);
	c[2] = (int)(r / L->T[1]);
}
static inline long up(const NLv *L, const int *c, int d){
	return c[d] + 1 < L->T[d] ? L->s[d] : -(long)(L->T[d] - 1)*L->s[d];
}
static inline long dn(const NLv *L, const int *c, int d){
	return c[d] > 0 ? -L->s[d] : (long)(L->T[d] - 1)*L->s[d];
}

/* one colour: points with (x+y+z) % 2 == pass (pass 0 = the reference's red) */
static void gs_pass(double *phi, const double *rho, const NLv *L, int pass, int nd3){
	long N = L->N;
	#pragma omp parallel for num_threads(orc_nthreads) if(N > ORC_PAR_MIN)
	for(long g = 0; g < N; g++){
		int c[3];
		coords(L, g, c);
		if(((c[0] + c[1] + c[2]) & 1) != pass) continue;
		double v;
		if(nd3){
			v = (1./6.)*(phi[g+up(L,c,0)] + phi[g+dn(L,c,0)] + phi[g+up(L,c,1)] + phi[g+dn(L,c,1)]
			           + phi[g+up(L,c,2)] + phi[g+dn(L,c,2)] + rho[g]);
		} else {
			v = 0;
			for(int d = 0; d < L->nd; d++) v += phi[g+up(L,c,d)] + phi[g+dn(L,c,d)];
			v += rho[g];
			v *= 1./(2*L->nd);
		}
		phi[g] = v;
	}
}

static void smooth(ONative *S, int q, int nIter, int nd3){
	for(int k = 0; k < nIter; k++){
		gs_pass(S->phi[q], S->rho[q], &S->L[q], 0, nd3);
		gs_pass(S->phi[q], S->rho[q], &S->L[q], 1, nd3);
	}
}

static double residual_at(const double *phi, const double *rho, const NLv *L, const int *c, long g){
	double r;
	if(L->nd == 3){
		r = -6.*phi[g];
		r += phi[g+up(L,c,0)] + phi[g+dn(L,c,0)] + phi[g+up(L,c,1)] + phi[g+dn(L,c,1)]
		   + phi[g+up(L,c,2)] + phi[g+dn(L,c,2)];
	} else {
		r = -(2.*L->nd)*phi[g];
		for(int d = 0; d < L->nd; d++) r += phi[g+up(L,c,d)] + phi[g+dn(L,c,d)];
	}
	return r + rho[g];
}

static void residual(ONative *S, int q){
	const NLv *L = &S->L[q];
	#pragma omp parallel for num_threads(orc_nthreads) if(L->N > ORC_PAR_MIN)
	for(long g = 0; g < L->N; g++){
		int c[3];
		coords(L, g, c);
		S->res[q][g] = residual_at(S->phi[q], S->rho[q], L, c, g);
	}
}

/* restriction of res[q] into rho[q+1], times 4 (native) */
static void restrict4(ONative *S, int q){
	const NLv *F = &S->L[q], *C = &S->L[q+1];
	const double *x = S->res[q];
	double *out = S->rho[q+1];
	int nd = F->nd;
	#pragma omp parallel for num_threads(orc_nthreads) if(C->N > ORC_PAR_MIN)
	for(long gc = 0; gc < C->N; gc++){
		int cc[3], cf[3] = {0, 0, 0};
		coords(C, gc, cc);
		long gf = 0;
		for(int d = 0; d < nd; d++){ cf[d] = 2*cc[d]; gf += (long)cf[d]*F->s[d]; }
		double v;
		if(S->nd3){
			v = (1./12.)*(6*x[gf] + x[gf+up(F,cf,0)] + x[gf+dn(F,cf,0)] + x[gf+up(F,cf,1)] + x[gf+dn(F,cf,1)]
			            + x[gf+up(F,cf,2)] + x[gf+dn(F,cf,2)]);
		} else {
			v = (2.*nd)*x[gf];
			for(int d = 0; d < nd; d++) v += x[gf+up(F,cf,d)] + x[gf+dn(F,cf,d)];
			v *= 1./(nd*4);
		}
		out[gc] = v*4.0;
	}
}

/* value of the prolongated coarse grid at fine point cf: interpolation
 * along the lowest odd dimension of values interpolated along the higher
 * ones -- the intermediate roundings of mgBilinProl's z, y, x passes */
static double prol(const double *cv, const NLv *C, const int *cf, int D){
	if(D == C->nd){
		long g = 0;
		for(int d = 0; d < C->nd; d++) g += (long)(cf[d] >> 1)*C->s[d];
		return cv[g];
	}
	if(!(cf[D] & 1)) return prol(cv, C, cf, D+1);
	int a[3] = {cf[0], cf[1], cf[2]}, b[3] = {cf[0], cf[1], cf[2]};
	a[D] = cf[D] - 1;
	b[D] = cf[D] + 1;
	if(b[D] >= 2*C->T[D]) b[D] -= 2*C->T[D];
	return 0.5*(prol(cv, C, a, D+1) + prol(cv, C, b, D+1));
}

static void prolong_add(ONative *S, int qf){
	const NLv *F = &S->L[qf], *C = &S->L[qf+1];
	#pragma omp parallel for num_threads(orc_nthreads) if(F->N > ORC_PAR_MIN)
	for(long g = 0; g < F->N; g++){
		int cf[3];
		coords(F, g, cf);
		S->phi[qf][g] += prol(S->phi[qf+1], C, cf, 0);
	}
}

static void neutralize(double *a, long N){
	double s = 0;
	for(long g = 0; g < N; g++) s += a[g];
	double mu = s/(double)N;
	#pragma omp parallel for num_threads(orc_nthreads) if(N > ORC_PAR_MIN)
	for(long g = 0; g < N; g++) a[g] = a[g] - mu;
}

static void vrec(ONative *S, OWorld *w, int q){
	int bottom = S->nLevels - 1;
	if(S->spectralCoarse && q == 1){
		/* multigrid:spectralCoarse: the level-1 correction solved exactly
		 * (pinc_mg.c vrec, rocFFT with the 7-point symbol on the device) */
		orc_discrete_poisson(S->L[1].nd, S->L[1].T, S->rho[1], S->phi[1]);
		prolong_add(S, 0);
		return;
	}
	int pre = w->preSmooth == ORC_SMOOTH_GS3D, post = w->postSmooth == ORC_SMOOTH_GS3D;
	int coarse = w->coarseSolv == ORC_SMOOTH_GS3D;
	if(q > 0) memset(S->phi[q], 0, S->L[q].N*sizeof(double));
	if(q == bottom){
		neutralize(S->rho[q], S->L[q].N);
		smooth(S, q, w->nCoarse, coarse);
		neutralize(S->phi[q], S->L[q].N);
		prolong_add(S, q-1);
		return;
	}
	/* level 0's rho and phi are neutralised once per solve
	 * (ow_native_solve); no neutralisation between the prolongation and the
	 * post-smoothing (pinc_mg.c vrec, k_mg_coarse) */
	if(q > 0) neutralize(S->rho[q], S->L[q].N);
	smooth(S, q, w->nPre, pre);
	residual(S, q);
	restrict4(S, q);
	vrec(S, w, q+1);
	smooth(S, q, w->nPost, post);
	if(q > 0) neutralize(S->phi[q], S->L[q].N);
	if(q > 0) prolong_add(S, q-1);
}

/* global index of rank-local true point p */
static long gidx(const OWorld *w, int r, const int *p, const int *Lg){
	const OMpi *m = &w->r[r].mpi;
	const OGrid *g = &w->r[r].rho;
	long gi = 0, s = 1;
	for(int d = 0; d < w->nDims; d++){ gi += (long)(m->subdomain[d]*g->trueSize[d+1] + p[d])*s; s *= Lg[d]; }
	return gi;
}
static long lidx(const OGrid *g, const int *p){
	long i = 0;
	for(int d = 0; d < g->rank - 1; d++) i += (long)(p[d] + g->nGhost[d+1])*g->sizeProd[d+1];
	return i;
}

static void gather_scatter(OWorld *w, double *rhoG, double *phiG, int scatter){
	int nd = w->nDims, Lg[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) Lg[d] = w->r[0].rho.trueSize[d+1]*w->r[0].mpi.nSubdomains[d];
	for(int r = 0; r < w->P; r++){
		OGrid *rho = &w->r[r].rho, *phi = &w->r[r].phi;
		int t[3] = {1, 1, 1};
		for(int d = 0; d < nd; d++) t[d] = rho->trueSize[d+1];
		for(int z = 0; z < t[2]; z++) for(int y = 0; y < t[1]; y++) for(int x = 0; x < t[0]; x++){
			int p[3] = {x, y, z};
			long gi = gidx(w, r, p, Lg), li = lidx(rho, p);
			if(scatter) phi->val[li] = phiG[gi];
			else { rhoG[gi] = rho->val[li]; phiG[gi] = phi->val[li]; }
		}
	}
}

void ow_native_solve(OWorld *w){
	ONative *S = w->native;
	gather_scatter(w, S->rho[0], S->phi[0], 0);
	long N = S->L[0].N;
	/* phi holds the last solution (the device's pinc_hip_extrapolate /
	 * pinc_hip_lincomb, same expressions) */
	const int role = S->extrap ? S->role : ON_GUESS_WARM;
	double *ph = S->phi[0];
	if(role == ON_GUESS_SERIES){
		if(S->nSeen >= 2){
			for(long g = 0; g < N; g++){ double p = ph[g]; ph[g] = 2.0*p - S->prev[g]; S->prev[g] = p; }
		} else if(S->nSeen == 1) memcpy(S->prev, ph, N*sizeof(double));
		if(S->nSeen < 2) S->nSeen++;
	} else if(role == ON_GUESS_FIRST && S->nSeen >= 2){
		for(long g = 0; g < N; g++) ph[g] = 2.0*S->A[g] + -1.0*S->B[g];
	} else if(role == ON_GUESS_SECOND && S->secondSpectral && S->nSeen >= 1){
		for(long g = 0; g < N; g++) S->rhoSave[g] = 1.0*S->rho[0][g] + -1.0*S->rhoSave[g];
		orc_discrete_poisson(S->L[0].nd, S->L[0].T, S->rhoSave, S->dphi);
		for(long g = 0; g < N; g++) ph[g] = 1.0*ph[g] + 1.0*S->dphi[g];
	} else if(role == ON_GUESS_SECOND && S->haveCorr){
		for(long g = 0; g < N; g++) ph[g] = 1.0*ph[g] + 1.0*S->D[g];
	}
	double barRes = 2.;
	long c = 0;
	w->mgHistN = 0;
	if(S->nLevels > 1) neutralize(S->rho[0], N);
	while(barRes > 1.E-10){
		vrec(S, w, 0);
		w->cycles++;
		double sum = 0;
		const NLv *L = &S->L[0];
		for(long g = 0; g < N; g++){
			int cc[3];
			coords(L, g, cc);
			double v = residual_at(S->phi[0], S->rho[0], L, cc, g);
			sum += v*v;
		}
		barRes = sqrt(sum/N);
		if(w->mgHistN < w->mgHistCap) w->mgHist[w->mgHistN] = barRes;
		w->mgHistN++;
		if(w->verbose && w->cycles % w->verbose == 0)
			fprintf(stderr, "[orc] native cycle %ld residual %.3e\n", (long)w->cycles, barRes);
		if(w->mgCap > 0 && ++c >= w->mgCap) break;
		if(!isfinite(barRes)) orc_die("native multigrid diverged (residual %g)", barRes);
	}
	if(S->nLevels > 1) neutralize(S->phi[0], N);
	if(role == ON_GUESS_FIRST){
		double *t = S->B; S->B = S->A; S->A = t;
		memcpy(S->A, ph, N*sizeof(double));
		if(S->secondSpectral) memcpy(S->rhoSave, S->rho[0], N*sizeof(double));
		if(S->nSeen < 2) S->nSeen++;
	} else if(role == ON_GUESS_SECOND && S->nSeen >= 1){
		for(long g = 0; g < N; g++) S->D[g] = 1.0*ph[g] + -1.0*S->A[g];
		S->haveCorr = 1;
	}
	if(S->objects) S->role = ON_GUESS_WARM;
	gather_scatter(w, NULL, S->phi[0], 1);
	OGrid *phi[256];
	for(int r = 0; r < w->P; r++) phi[r] = &w->r[r].phi;
	ow_halo(w, phi, OP_SET, TOHALO);
	w->solves++;
}
