/*
 * orc_mg.c -- TEST INFRASTRUCTURE (oracle).  Restates the multigrid Poisson
 * solver of src/multigrid.c (and the 1-D spectral solver of spectral.c):
 *   ow_mg_alloc        mgAllocSolver/mgAlloc/mgAllocSubGrids  multigrid.c:128-214,297-384
 *   omg_gs_pass(nd3=1) mgGS3D  red (j+k+l odd) then black, the sweep covers
 *                      the x/y ghost columns of every true z layer   multigrid.c:683-767
 *   omg_gs_pass(nd3=0) mgGSND  true points only; first pass holds   multigrid.c:553-621
 *                      (1,..,1), phi = (sum_d (f+ + f-) + rho)/(2D)
 *   omg_residual       mgResidual + gFinDiff2nd3D/ND    multigrid.c:1385-1403
 *   omg_restrict       mgHalfRestrict3D (1/12) / ND (1/(4D) over the whole
 *                      coarse array)                    multigrid.c:844-1022
 *   omg_inject +       mgBilinProl3D / mgBilinProlND: inject at odd fine
 *   omg_prolong_dim    points, then interpolate z, y, x with a TOHALO of
 *                      that dimension before each pass  multigrid.c:1024-1238
 *   vrec               mgVRecursiveInner                multigrid.c:1496-1556
 *   ow_mg_solve        mgSolveRaw (RMS residual <= 1e-10, >= 1 cycle)
 *                                                       multigrid.c:1688-1724
 *   ow_spectral_solve  sSolve (1-D): phi_n = rho_n*(N/2 pi n)^2/N, DC = 0
 *                                                       spectral.c:14-115
 * The prolongation writes of the reference that land in ghost cells (and are
 * overwritten by a halo exchange before any true point reads them) are not
 * reproduced; every true-point value is.  Coarse phi levels persist between
 * cycles and time steps (warm start), as in the reference.
 */
#include "orc.h"
#include <math.h>

void ow_mg_alloc(OWorld *w){
	int L = w->nLevels;
	for(int r = 0; r < w->P; r++){
		ORank *R = &w->r[r];
		OMg *m[3] = {&R->mgRho, &R->mgPhi, &R->mgRes};
		OGrid *g0[3] = {&R->rho, &R->phi, &R->res};
		for(int d = 1; d < R->rho.rank; d++)
			if(R->rho.trueSize[d] % (1 << L))
				orc_die("All elements in grid:trueSize must be a multiple of 2^mgLevels=%d", 1 << L);
		for(int k = 0; k < 3; k++){
			m[k]->nLevels = L;
			m[k]->grids = calloc(L, sizeof(OGrid*));
			m[k]->grids[0] = g0[k];
			for(int q = 1; q < L; q++){
				m[k]->grids[q] = calloc(1, sizeof(OGrid));
				og_alloc_sub(m[k]->grids[q], g0[k], q);
			}
		}
	}
}

/* One colour of red-black Gauss-Seidel.  pass 0 updates the colour of the
 * point (1,..,1), pass 1 the other colour.  Points are visited in memory
 * order exactly as the reference visits them. */
void omg_gs_pass(OGrid *phi, const OGrid *rho, int pass, int nd3){
	const long *sp = phi->sizeProd;
	double *f = phi->val;
	const double *q = rho->val;
	int rank = phi->rank;
	if(nd3){
		double coeff = 1./6.;
		int parity = (pass == 0) ? 1 : 0; /* red: j+k+l odd */
		/* points of one colour only read the other colour: any visiting
		 * order gives the same values */
		#pragma omp parallel for num_threads(orc_nthreads) if(sp[4] > ORC_PAR_MIN)
		for(int l = 1; l <= phi->trueSize[3]; l++)
			for(int k = 0; k < phi->size[2]; k++)
				for(int j = (k + l + parity) & 1; j < phi->size[1]; j += 2){
					long g = j + k*sp[2] + l*sp[3];
					f[g] = coeff*(f[g+1] + f[g-1] + f[g+sp[2]] + f[g-sp[2]]
					            + f[g+sp[3]] + f[g-sp[3]] + q[g]);
				}
		return;
	}
	int nd = rank - 1;
	double coeff = 1./(2*(rank-1));
	int want = (nd + pass) & 1; /* parity of the coordinate sum */
	int T[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) T[d] = phi->trueSize[d+1];
	#pragma omp parallel for num_threads(orc_nthreads) if(sp[rank] > ORC_PAR_MIN)
	for(int z = 1; z <= (nd > 2 ? T[2] : 1); z++)
		for(int y = 1; y <= (nd > 1 ? T[1] : 1); y++)
			for(int x = 1; x <= T[0]; x++){
				int csum = x + (nd > 1 ? y : 0) + (nd > 2 ? z : 0);
				if((csum & 1) != want) continue;
				long g = x + (nd > 1 ? y*sp[2] : 0) + (nd > 2 ? z*sp[3] : 0);
				double v = 0;
				for(int r = 1; r <= nd; r++) v += f[g+sp[r]] + f[g-sp[r]];
				v += q[g];
				v *= coeff;
				f[g] = v;
			}
}

void omg_residual(OGrid *res, const OGrid *rho, const OGrid *phi){
	og_findiff2nd(res, phi);
	long n = res->sizeProd[res->rank];
	for(long g = 0; g < n; g++) res->val[g] += rho->val[g];
}

void omg_restrict(const OGrid *fine, OGrid *coarse, int nd3){
	const long *fs = fine->sizeProd, *cs = coarse->sizeProd;
	const double *f = fine->val;
	double *c = coarse->val;
	int rank = fine->rank, nd = rank - 1;
	int T[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) T[d] = coarse->trueSize[d+1];
	if(nd3){
		double coeff = 1./12.;
		#pragma omp parallel for num_threads(orc_nthreads) if(cs[rank] > ORC_PAR_MIN)
		for(int l = 1; l <= T[2]; l++)
			for(int k = 1; k <= T[1]; k++)
				for(int j = 1; j <= T[0]; j++){
					long gf = (2*j-1) + (2*k-1)*fs[2] + (2*l-1)*fs[3];
					long gc = j + k*cs[2] + l*cs[3];
					c[gc] = coeff*(6*f[gf] + f[gf+1] + f[gf-1] + f[gf+fs[2]] + f[gf-fs[2]]
					             + f[gf+fs[3]] + f[gf-fs[3]]);
				}
		return;
	}
	double c0 = 2.*nd;
	#pragma omp parallel for num_threads(orc_nthreads) if(cs[rank] > ORC_PAR_MIN)
	for(int l = 1; l <= (nd > 2 ? T[2] : 1); l++)
		for(int k = 1; k <= (nd > 1 ? T[1] : 1); k++)
			for(int j = 1; j <= T[0]; j++){
				long gf = (2*j-1) + (nd > 1 ? (2*k-1)*fs[2] : 0) + (nd > 2 ? (2*l-1)*fs[3] : 0);
				long gc = j + (nd > 1 ? k*cs[2] : 0) + (nd > 2 ? l*cs[3] : 0);
				double v = c0*f[gf];
				for(int r = 1; r <= nd; r++) v += f[gf+fs[r]] + f[gf-fs[r]];
				c[gc] = v;
			}
	double coeff = 1./((rank-1)*4);
	long n = cs[rank];
	for(long g = 0; g < n; g++) c[g] *= coeff;
}

void omg_inject(OGrid *fine, const OGrid *coarse){
	const long *fs = fine->sizeProd, *cs = coarse->sizeProd;
	int nd = fine->rank - 1;
	int T[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) T[d] = coarse->trueSize[d+1];
	#pragma omp parallel for num_threads(orc_nthreads) if(cs[fine->rank] > ORC_PAR_MIN)
	for(int l = 1; l <= T[2]; l++)
		for(int k = 1; k <= T[1]; k++)
			for(int j = 1; j <= T[0]; j++){
				long gf = (2*j-1) + (nd > 1 ? (2*k-1)*fs[2] : 0) + (nd > 2 ? (2*l-1)*fs[3] : 0);
				long gc = j + (nd > 1 ? k*cs[2] : 0) + (nd > 2 ? l*cs[3] : 0);
				fine->val[gf] = coarse->val[gc];
			}
}

/* Linear interpolation along dimension r (1-based): points whose coordinate
 * in r is even, whose coordinates in dimensions below r are odd, and any
 * coordinate in dimensions above r. */
void omg_prolong_dim(OGrid *fine, int r){
	const long *fs = fine->sizeProd;
	int nd = fine->rank - 1;
	int T[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) T[d] = fine->trueSize[d+1];
	/* written points are even along r and read odd neighbours along r only */
	#pragma omp parallel for num_threads(orc_nthreads) if(fs[fine->rank] > ORC_PAR_MIN)
	for(int z = 1; z <= T[2]; z++)
		for(int y = 1; y <= T[1]; y++)
			for(int x = 1; x <= T[0]; x++){
				int c[4] = {0, x, y, z};
				int ok = 1;
				for(int d = 1; d <= nd; d++){
					if(d == r && (c[d] & 1)) ok = 0;
					if(d < r && !(c[d] & 1)) ok = 0;
				}
				if(!ok) continue;
				long g = 0;
				for(int d = 1; d <= nd; d++) g += c[d]*fs[d];
				fine->val[g] = 0.5*(fine->val[g+fs[r]] + fine->val[g-fs[r]]);
			}
}

/* ------------------------------------------------------ world-level MG -- */
static void collect(OWorld *w, OMg *(*sel)(ORank*), int level, OGrid **out){
	for(int r = 0; r < w->P; r++) out[r] = sel(&w->r[r])->grids[level];
}
static OMg *selRho(ORank *R){ return &R->mgRho; }
static OMg *selPhi(ORank *R){ return &R->mgPhi; }
static OMg *selRes(ORank *R){ return &R->mgRes; }

static void ow_gs(OWorld *w, int level, int nCycles, int which){
	OGrid *phi[256], *rho[256];
	collect(w, selPhi, level, phi);
	collect(w, selRho, level, rho);
	int nd3 = (which == ORC_SMOOTH_GS3D);
	for(int c = 0; c < nCycles; c++){
		for(int pass = 0; pass < 2; pass++){
			for(int r = 0; r < w->P; r++) omg_gs_pass(phi[r], rho[r], pass, nd3);
			ow_halo(w, phi, OP_SET, TOHALO);
			ow_neutralize(w, phi);
		}
	}
}

static void ow_prolong(OWorld *w, int coarseLevel){
	OGrid *fine[256], *coarse[256];
	collect(w, selRes, coarseLevel-1, fine);
	collect(w, selPhi, coarseLevel, coarse);
	for(int r = 0; r < w->P; r++) omg_inject(fine[r], coarse[r]);
	for(int d = fine[0]->rank-1; d > 0; d--){
		ow_halo_dim(w, fine, d, OP_SET, TOHALO);
		for(int r = 0; r < w->P; r++) omg_prolong_dim(fine[r], d);
	}
}

static void vrec(OWorld *w, int level, int bottom, int top){
	OGrid *phi[256], *rho[256], *res[256];
	collect(w, selPhi, level, phi);
	collect(w, selRho, level, rho);
	collect(w, selRes, level, res);
	if(level == bottom){
		ow_halo(w, phi, OP_SET, TOHALO);
		ow_halo(w, rho, OP_SET, TOHALO);
		ow_neutralize(w, rho);
		ow_gs(w, level, w->nCoarse, w->coarseSolv);
		ow_neutralize(w, phi);
		ow_prolong(w, level);
		return;
	}
	ow_halo(w, rho, OP_SET, TOHALO);
	ow_neutralize(w, rho);
	ow_gs(w, level, w->nPre, w->preSmooth);
	for(int r = 0; r < w->P; r++) omg_residual(res[r], rho[r], phi[r]);
	ow_halo(w, res, OP_SET, TOHALO);
	for(int r = 0; r < w->P; r++)
		omg_restrict(res[r], w->r[r].mgRho.grids[level+1], w->restrictor == ORC_RESTR_3D);
	vrec(w, level+1, bottom, top);
	for(int r = 0; r < w->P; r++) og_addto(phi[r], res[r]);
	ow_halo(w, phi, OP_SET, TOHALO);
	ow_neutralize(w, phi);
	ow_gs(w, level, w->nPost, w->postSmooth);
	ow_neutralize(w, phi);
	if(level > top) ow_prolong(w, level);
}

void ow_mg_solve(OWorld *w){
	int bottom = w->nLevels - 1;
	w->solves++;
	if(w->nLevels > 1){
		double barRes = 2.;
		OGrid *rho[256], *phi[256], *res[256];
		collect(w, selRho, 0, rho);
		collect(w, selPhi, 0, phi);
		collect(w, selRes, 0, res);
		long N = og_tot_truesize(rho[0], &w->r[0].mpi);
		long c = 0;
		w->mgHistN = 0;
		while(barRes > 1.E-10){
			vrec(w, 0, bottom, 0);
			w->cycles++;
			for(int r = 0; r < w->P; r++) omg_residual(res[r], rho[r], phi[r]);
			ow_halo(w, res, OP_SET, TOHALO);
			double sum = 0;
			for(int r = 0; r < w->P; r++){ og_square(res[r]); sum += og_sum_true(res[r]); }
			barRes = sqrt(sum/N);
			if(w->mgHistN < w->mgHistCap) w->mgHist[w->mgHistN] = barRes;
			w->mgHistN++;
			if(w->mgCap > 0 && ++c >= w->mgCap) break;
			if(w->verbose && w->cycles % w->verbose == 0)
				fprintf(stderr, "[orc] cycle %ld residual %.3e\n", (long)w->cycles, barRes);
		}
	} else {
		OGrid *rho[256], *phi[256];
		collect(w, selRho, 0, rho);
		collect(w, selPhi, 0, phi);
		for(int c = 0; c < w->mgCycles; c++){
			ow_halo(w, rho, OP_SET, TOHALO);
			ow_neutralize(w, rho);
			ow_gs(w, 0, w->nCoarse, w->coarseSolv);
		}
	}
}

/* 1-D spectral Poisson solve by direct DFT (N is small in the 1-D configs).
 * FFTW's r2c/c2r are unnormalised; the factor (N/2 pi n)^2/N carries the
 * 1/N.  c2r ignores the imaginary part of the DC and Nyquist bins. */
static void ow_spectral_solve_nd(OWorld *w);

void ow_spectral_solve(OWorld *w){
	if(w->nDims != 1 || w->P != 1){ ow_spectral_solve_nd(w); return; }
	OGrid *rho = &w->r[0].rho, *phi = &w->r[0].phi;
	int N = rho->trueSize[1];
	int M = N/2 + 1;
	double *re = calloc(M, sizeof(double)), *im = calloc(M, sizeof(double));
	int g = rho->nGhost[1];
	for(int n = 0; n < M; n++){
		double a = 0, b = 0;
		for(int x = 0; x < N; x++){
			double t = -2.0*M_PI*(double)n*x/N;
			a += rho->val[g+x]*cos(t);
			b += rho->val[g+x]*sin(t);
		}
		re[n] = a; im[n] = b;
	}
	re[0] = im[0] = 0;
	for(int n = 1; n < M; n++){ re[n] *= w->spectralFactor[n]; im[n] *= w->spectralFactor[n]; }
	for(int x = 0; x < N; x++){
		double v = re[0];
		for(int n = 1; n < M; n++){
			double t = 2.0*M_PI*(double)n*x/N;
			double term = re[n]*cos(t) - im[n]*sin(t);
			if(2*n == N) v += term; else v += 2*term;
		}
		phi->val[g+x] = v;
	}
	free(re); free(im);
	w->solves++;
}

/* N-D extension of sSolve (the reference is 1-D only, spectral.c:80-89):
 * phi = IDFT(DFT(rho) * f(k)), f = 1/|k|^2/N with k_d = 2 pi n_d/N_d over the
 * signed frequencies, f(0) = 0, on the global periodic grid gathered from
 * every emulated rank's true nodes.  The full complex spectrum is used, one
 * naive DFT along each dimension (separable), which in exact arithmetic
 * equals the r2c/c2r pair of the build.  Ghosts are left to the TOHALO that
 * follows every solve (main.c:240). */
static void dft_axis(double *re, double *im, const int *L, int axis, int sign){
	long stride = 1;
	for(int d = 0; d < axis; d++) stride *= L[d];
	int n = L[axis];
	long outer = 1;
	for(int d = 0; d < 3; d++) if(d != axis) outer *= L[d];
	double *cr = malloc(n*sizeof(double)), *ci = malloc(n*sizeof(double));
	for(int k = 0; k < n; k++){
		cr[k] = cos(2.0*M_PI*k/n);
		ci[k] = sign*sin(2.0*M_PI*k/n);
	}
	/* lines are independent: OpenMP over them, bit-identical for any count */
	#pragma omp parallel
	{
	double *tr = malloc(n*sizeof(double)), *ti = malloc(n*sizeof(double));
	#pragma omp for schedule(static)
	for(long o = 0; o < outer; o++){
		/* base index of the line: decompose o over the other axes */
		long base = 0, r = o, s = 1;
		for(int d = 0; d < 3; d++){
			if(d == axis){ s *= L[d]; continue; }
			base += (r % L[d])*s;
			r /= L[d];
			s *= L[d];
		}
		for(int k = 0; k < n; k++){
			double a = 0, b = 0;
			for(int x = 0; x < n; x++){
				int t = (int)(((long)k*x) % n);
				double vr = re[base + x*stride], vi = im[base + x*stride];
				a += vr*cr[t] - vi*ci[t];
				b += vr*ci[t] + vi*cr[t];
			}
			tr[k] = a; ti[k] = b;
		}
		for(int k = 0; k < n; k++){ re[base + k*stride] = tr[k]; im[base + k*stride] = ti[k]; }
	}
	free(tr); free(ti);
	}
	free(cr); free(ci);
}

/* phi = the exact solution of the multigrid's discrete Poisson problem
 * -(sum of the 2 nd neighbours - 2 nd phi) = rho on a global periodic grid L
 * (x fastest), DC dropped: phi = IDFT(DFT(rho) / sum_d (2 - 2 cos(2 pi
 * n_d/L_d)) / N), the symbol of the device's pinc_hip_fft_set_symbol(plan,
 * 1) (objects:secondGuess = spectral) */
void orc_discrete_poisson(int nd, const int *Lin, const double *rho, double *phi){
	int L[3] = {1, 1, 1};
	for(int d = 0; d < nd; d++) L[d] = Lin[d];
	long N = (long)L[0]*L[1]*L[2];
	double *re = malloc(N*sizeof(double)), *im = calloc(N, sizeof(double));
	memcpy(re, rho, N*sizeof(double));
	for(int d = 0; d < nd; d++) dft_axis(re, im, L, d, -1);
	for(long i = 0; i < N; i++){
		long r = i;
		double s = 0;
		for(int d = 0; d < nd; d++){
			int n = (int)(r % L[d]);
			r /= L[d];
			if(n > L[d]/2) n -= L[d];
			s += 2.0 - 2.0*cos(2*M_PI*n/L[d]);
		}
		double f = i ? 1.0/s/N : 0.0;
		re[i] *= f; im[i] *= f;
	}
	for(int d = 0; d < nd; d++) dft_axis(re, im, L, d, +1);
	memcpy(phi, re, N*sizeof(double));
	free(re); free(im);
}

/* global index <-> rank-local padded index (x fastest, ghosts g per side) */
static long local_index(const OGrid *g, const int *p){
	long i = 0;
	for(int d = 0; d < g->rank - 1; d++) i += (long)(p[d] + g->nGhost[d+1])*g->sizeProd[d+1];
	return i;
}

static void ow_spectral_solve_nd(OWorld *w){
	int nd = w->nDims;
	int L[3] = {1, 1, 1};
	const OMpi *m0 = &w->r[0].mpi;
	for(int d = 0; d < nd; d++) L[d] = w->r[0].rho.trueSize[d+1]*m0->nSubdomains[d];
	long N = (long)L[0]*L[1]*L[2];
	double *re = calloc(N, sizeof(double)), *im = calloc(N, sizeof(double));
	for(int r = 0; r < w->P; r++){
		const OGrid *rho = &w->r[r].rho;
		const OMpi *m = &w->r[r].mpi;
		int t[3] = {1, 1, 1};
		for(int d = 0; d < nd; d++) t[d] = rho->trueSize[d+1];
		for(int z = 0; z < t[2]; z++) for(int y = 0; y < t[1]; y++) for(int x = 0; x < t[0]; x++){
			int p[3] = {x, y, z};
			long gi = 0, s = 1;
			for(int d = 0; d < nd; d++){ gi += (long)(m->subdomain[d]*t[d] + p[d])*s; s *= L[d]; }
			re[gi] = rho->val[local_index(rho, p)];
		}
	}
	for(int d = 0; d < nd; d++) dft_axis(re, im, L, d, -1);
	for(long i = 0; i < N; i++){
		long r = i;
		double k2 = 0;
		for(int d = 0; d < nd; d++){
			int n = (int)(r % L[d]);
			r /= L[d];
			if(n > L[d]/2) n -= L[d];
			double k = 2*M_PI*n/L[d];
			k2 += k*k;
		}
		double f = 0;
		if(i){ f = 1.0/k2; f /= N; }
		re[i] *= f; im[i] *= f;
	}
	for(int d = 0; d < nd; d++) dft_axis(re, im, L, d, +1);
	for(int r = 0; r < w->P; r++){
		OGrid *phi = &w->r[r].phi;
		const OMpi *m = &w->r[r].mpi;
		int t[3] = {1, 1, 1};
		for(int d = 0; d < nd; d++) t[d] = phi->trueSize[d+1];
		for(int z = 0; z < t[2]; z++) for(int y = 0; y < t[1]; y++) for(int x = 0; x < t[0]; x++){
			int p[3] = {x, y, z};
			long gi = 0, s = 1;
			for(int d = 0; d < nd; d++){ gi += (long)(m->subdomain[d]*t[d] + p[d])*s; s *= L[d]; }
			phi->val[local_index(phi, p)] = re[gi];
		}
	}
	free(re); free(im);
	w->solves++;
}
