/*
 * orc_grid.c -- TEST INFRASTRUCTURE (oracle).  Restates the grid glue of
 * src/grid.c that runs inside a PIC timestep:
 *   og_alloc            gAlloc            grid.c:413-500
 *   og_alloc_sub        mgAllocSubGrids   multigrid.c:128-214
 *   og_mul/zero/...     gMul/gZero/...    grid.c:668-802
 *   og_sum_true         gSumTruegrid      grid.c:804-847 (nested row/plane sums)
 *   og_pot_energy_inner gPotEnergyInner   grid.c:1295-1321
 *   og_findiff1st       gFinDiff1st       grid.c:226-261
 *   og_findiff2nd       gFinDiff2nd3D/ND  grid.c:264-334
 *   ow_halo(_dim)       gHaloOp(Dim)      grid.c:340-406 + get/set/addSlice 72-147
 *   ow_neutralize       gNeutralizeGrid   grid.c:730-779
 * Floating-point expressions keep the reference's association order.
 */
#include "orc.h"

static void cumprod(const int *a, long *res, int n){
	res[0] = 1;
	for(int i = 0; i < n; i++) res[i+1] = res[i]*a[i];
}

void og_alloc(OGrid *g, const OIni *ini, int nValues){
	int nDims = oini_int(ini, "grid:nDims");
	int *ts = oini_intarr(ini, "grid:trueSize", nDims);
	int *ng = oini_intarr(ini, "grid:nGhostLayers", 2*nDims);
	memset(g, 0, sizeof(*g));
	int rank = nDims + 1;
	g->rank = rank;
	if(nValues < 0) nValues = nDims;
	g->size[0] = g->trueSize[0] = nValues;
	g->nGhost[0] = g->nGhost[rank] = 0;
	for(int d = 1; d < rank; d++){
		g->trueSize[d] = ts[d-1];
		g->nGhost[d] = ng[d-1];
		g->nGhost[d+rank] = ng[d+nDims-1];
		g->size[d] = g->trueSize[d] + g->nGhost[d] + g->nGhost[d+rank];
	}
	cumprod(g->size, g->sizeProd, rank);
	/* The reference mallocs val uninitialised; fresh pages read as zero. */
	g->val = calloc(g->sizeProd[rank], sizeof(double));
	free(ts); free(ng);
}

void og_alloc_sub(OGrid *g, const OGrid *fine, int q){
	memset(g, 0, sizeof(*g));
	int rank = fine->rank;
	g->rank = rank;
	g->size[0] = g->trueSize[0] = fine->trueSize[0];
	for(int d = 0; d < 2*rank; d++) g->nGhost[d] = fine->nGhost[d];
	for(int d = 1; d < rank; d++){
		g->trueSize[d] = fine->trueSize[d] >> q;
		g->size[d] = g->trueSize[d] + g->nGhost[d] + g->nGhost[rank+d];
	}
	cumprod(g->size, g->sizeProd, rank);
	g->val = calloc(g->sizeProd[rank], sizeof(double));
}

void og_free(OGrid *g){ free(g->val); g->val = NULL; }

void og_zero(OGrid *g){ memset(g->val, 0, g->sizeProd[g->rank]*sizeof(double)); }

int orc_nthreads = 1;

void og_mul(OGrid *g, double num){
	long n = g->sizeProd[g->rank];
	#pragma omp parallel for num_threads(orc_nthreads) if(n > ORC_PAR_MIN)
	for(long p = 0; p < n; p++) g->val[p] *= num;
}

void og_sub(OGrid *g, double num){
	long n = g->sizeProd[g->rank];
	#pragma omp parallel for num_threads(orc_nthreads) if(n > ORC_PAR_MIN)
	for(long p = 0; p < n; p++) g->val[p] -= num;
}

void og_addto(OGrid *res, const OGrid *add){
	long n = res->sizeProd[res->rank];
	#pragma omp parallel for num_threads(orc_nthreads) if(n > ORC_PAR_MIN)
	for(long p = 0; p < n; p++) res->val[p] += add->val[p];
}

void og_square(OGrid *g){
	long n = g->sizeProd[g->rank];
	#pragma omp parallel for num_threads(orc_nthreads) if(n > ORC_PAR_MIN)
	for(long p = 0; p < n; p++) g->val[p] = g->val[p]*g->val[p];
}

/* Nested sum over true points: rows are summed first, then rows into planes,
 * planes into the volume, each partial starting from zero (grid.c:804-831). */
static double sum_level(const OGrid *g, int d, long base){
	double s = 0.;
	long lo = g->nGhost[d];
	if(d == 1){
		for(int j = 0; j < g->trueSize[1]; j++) s += g->val[base + lo + j];
	} else {
		for(int j = 0; j < g->trueSize[d]; j++)
			s += sum_level(g, d-1, base + (lo + j)*g->sizeProd[d]);
	}
	return s;
}

double og_sum_true(const OGrid *g){ return sum_level(g, g->rank-1, 0); }

static double pe_level(const OGrid *rho, const OGrid *phi, int d, long base){
	double e = 0.;
	long lo = rho->nGhost[d];
	if(d == 1){
		for(int j = 0; j < rho->trueSize[1]; j++)
			e += rho->val[base + lo + j]*phi->val[base + lo + j];
	} else {
		for(int j = 0; j < rho->trueSize[d]; j++)
			e += pe_level(rho, phi, d-1, base + (lo + j)*rho->sizeProd[d]);
	}
	return e;
}

double og_pot_energy_inner(const OGrid *rho, const OGrid *phi){
	return pe_level(rho, phi, rho->rank-1, 0);
}

long og_tot_truesize(const OGrid *g, const OMpi *mpi){
	long t = 1;
	for(int r = 1; r < g->rank; r++) t *= (long)mpi->nSubdomains[r-1]*g->trueSize[r];
	return t;
}

/* E_d = 0.5*(phi[g+s_d]-phi[g-s_d]) over the linear interior range. */
void og_findiff1st(const OGrid *scalar, OGrid *field){
	int rank = scalar->rank;
	const long *sp = scalar->sizeProd;
	long fstride = field->sizeProd[1];
	long start = 0;
	for(int d = 1; d < rank; d++) start += sp[d];
	long end = sp[rank] - start;
	for(int d = 1; d < rank; d++){
		#pragma omp parallel for num_threads(orc_nthreads) if(end - start > ORC_PAR_MIN)
		for(long g = start; g < end; g++)
			field->val[g*fstride + (d-1)] = 0.5*(scalar->val[g + sp[d]] - scalar->val[g - sp[d]]);
	}
}

/* Laplacian with the reference's association: 3-D sums the six neighbours
 * left to right before adding to -6*phi; N-D adds each +-pair in turn. */
void og_findiff2nd(OGrid *res, const OGrid *phi){
	int rank = phi->rank;
	const long *sp = phi->sizeProd;
	const double *p = phi->val;
	long g0 = 0;
	for(int d = 1; d < rank; d++) g0 += sp[d];
	if(rank == 4){
		long end = sp[rank] - 2*g0;
		#pragma omp parallel for num_threads(orc_nthreads) if(end > ORC_PAR_MIN)
		for(long q = 0; q < end; q++){
			long g = g0 + q;
			double r = -6.*p[g];
			r += p[g+sp[1]] + p[g-sp[1]] + p[g+sp[2]] + p[g-sp[2]] + p[g+sp[3]] + p[g-sp[3]];
			res->val[g] = r;
		}
	} else {
		long end = sp[rank] - 2*g0;
		double coeff = 2.*(rank-1);
		#pragma omp parallel for num_threads(orc_nthreads) if(end > ORC_PAR_MIN)
		for(long q = 0; q < end + 1; q++){
			long g = g0 + q;
			double r = -coeff*p[g];
			for(int k = 1; k < rank; k++) r += p[g+sp[k]] + p[g-sp[k]];
			res->val[g] = r;
		}
	}
}

/* ------------------------------------------------------------- halo --- */
static long slice_len(const OGrid *g, int d){ return g->sizeProd[g->rank]/g->size[d]; }

static void get_slice(double *s, const OGrid *g, int d, int offset){
	long inner = g->sizeProd[d], outer = g->sizeProd[g->rank]/g->sizeProd[d+1];
	long k = 0;
	for(long o = 0; o < outer; o++){
		const double *v = g->val + o*g->sizeProd[d+1] + offset*g->sizeProd[d];
		for(long i = 0; i < inner; i++) s[k++] = v[i];
	}
}

static void put_slice(const double *s, OGrid *g, int d, int offset, int op){
	long inner = g->sizeProd[d], outer = g->sizeProd[g->rank]/g->sizeProd[d+1];
	long k = 0;
	for(long o = 0; o < outer; o++){
		double *v = g->val + o*g->sizeProd[d+1] + offset*g->sizeProd[d];
		if(op == OP_ADD) for(long i = 0; i < inner; i++) v[i] += s[k++];
		else for(long i = 0; i < inner; i++) v[i] = s[k++];
	}
}

static int nbr_rank(const OMpi *m, int dd, int dir){
	int first = m->mpiRank - m->subdomain[dd]*m->nSubdomainsProd[dd];
	int n = m->nSubdomains[dd];
	return first + ((m->subdomain[dd] + dir + n) % n)*m->nSubdomainsProd[dd];
}

void ow_halo_dim(OWorld *w, OGrid **grids, int d, int op, int dir){
	int P = w->P;
	const OGrid *g0 = grids[0];
	int upTake = g0->size[d] - 2 + dir, upPlace = g0->size[d] - 1 - dir;
	int loTake = 1 - dir, loPlace = dir;
	long n = slice_len(g0, d);
	double *buf = malloc((size_t)P*n*sizeof(double));
	/* send upper, receive from lower (tag 1) */
	for(int r = 0; r < P; r++) get_slice(buf + (long)r*n, grids[r], d, upTake);
	for(int r = 0; r < P; r++){
		int src = nbr_rank(&w->r[r].mpi, d-1, -1);
		put_slice(buf + (long)src*n, grids[r], d, loPlace, op);
	}
	/* send lower, receive from upper (tag 0) */
	for(int r = 0; r < P; r++) get_slice(buf + (long)r*n, grids[r], d, loTake);
	for(int r = 0; r < P; r++){
		int src = nbr_rank(&w->r[r].mpi, d-1, +1);
		put_slice(buf + (long)src*n, grids[r], d, upPlace, op);
	}
	free(buf);
}

void ow_halo(OWorld *w, OGrid **grids, int op, int dir){
	for(int d = 1; d < grids[0]->rank; d++) ow_halo_dim(w, grids, d, op, dir);
}

void ow_neutralize(OWorld *w, OGrid **grids){
	double tot = 0.;
	for(int r = 0; r < w->P; r++) tot += og_sum_true(grids[r]);
	const OGrid *g = grids[0];
	int prod = 1;
	for(int d = 1; d < g->rank; d++) prod *= g->trueSize[d];
	double avg = tot/((double)prod*w->P);
	for(int r = 0; r < w->P; r++) og_sub(grids[r], avg);
}
