/*
 * orc_obj.c -- TEST INFRASTRUCTURE (CPU checker, never shipped): plain-C
 * restatement of the reference's immersed-object path, object.c (SURVEY.md
 * 8(f) item 1, config C5), for one subdomain (P = 1).
 *
 *   oo_create        oFillLookupTables (object.c:111-160) and
 *                    oFindObjectSurfaceNodes (object.c:368-458) on a node
 *                    mask with periodic ghosts (oReadH5 + halo)
 *   oo_capacitance   oComputeCapacitanceMatrix (object.c:163-298): one
 *                    solve per surface node with a unit charge there, the
 *                    potentials at the surface nodes as a column, LU inverse
 *                    (gsl_linalg_LU_decomp/invert -> Gauss-Jordan with
 *                    partial pivoting here), 1/sum of the inverse
 *   oo_apply         oApplyCapacitanceMatrix (object.c:301-366): object
 *                    potential phi_c, surface correction charge, added to rho
 *   oo_collect       oCollectObjectCharge (object.c:460-515)
 *   oo_step          main.c:197-274 with the object calls (main.c:222-238)
 *
 * The reference does not compile, so this follows the
 * source text, with three defects corrected and named here:
 *   - object.c:499 calls pCut(pop, s, p, ...) with the NODE index p where the
 *     particle's position offset i*nDims is meant; here particle i is cut;
 *   - the swapped-in last particle is re-tested (the reference's loop moves
 *     on, leaving it inside the object for a step);
 *   - object.c:243 resets mgRho at lookupSurf[inode] without the object's
 *     offset (wrong node for every object but the first);
 *   - object.c:476-478 spreads object a's collected charge with
 *     invNrSurfNod[a] = 1/lookupSurfaceOffset[a+1], the CUMULATIVE surface
 *     count of objects 0..a (the commented-out line above it divides by the
 *     total), so every object after the first loses part of its charge;
 *     here the divisor is object a's own surface count (the reference's
 *     form is kept behind oo_set_reference_divisor for the test that pins
 *     the difference, tests/test_oracle_objects.py);
 *   - the reference spreads each rank's own count over that rank's own
 *     surface nodes, with no reduction; the build sums the count over the
 *     ranks and spreads it over all of the object's surface nodes (the same
 *     for an object inside one subdomain; this checker has one).
 * The spreading keeps the reference's expression, count * (1.0/divisor).
 * Parity of a build against this restatement is therefore parity against
 * the algorithm, pinned by its invariants (tests/test_oracle_objects.py):
 * after the correction the surface is an equipotential at phi_c, the
 * correction charge sums to zero, collected charge is conserved.
 */
#include "orc.h"
#include <math.h>

struct OObj {
	int nObjects;
	int refDivisor;       /* 1: object.c:476-478's cumulative divisor (tests only) */
	long nNodes;          /* nodes of the padded grid */
	double *mask;         /* node values (object id, 0 = vacuum) */
	int *objOfNode;       /* interior object of a true node (0 = none) */
	long *interior, *interiorOff;
	long *surface, *surfaceOff;
	double *capInv;       /* per object: inverse of the surface response matrix, row-major */
	long *capOff;
	double *capSum;       /* 1 / sum of the inverse */
	OGrid rhoObj;
	double *collected;    /* charge collected so far, per object */
	int haveCap;
};

static int is_ghost(const OGrid *g, long node) {
	int nd = g->rank - 1;
	for (int d = nd; d >= 1; d--) {
		long c = (node / g->sizeProd[d]) % g->size[d];
		if (c < g->nGhost[d] || c >= g->size[d] - g->nGhost[g->rank + d]) return 1;
	}
	return 0;
}

/* periodic ghost fill of a node-valued mask (the reference halos it) */
static void fill_ghosts(const OGrid *g, double *v) {
	int nd = g->rank - 1;
	for (long node = 0; node < g->sizeProd[g->rank]; node++) {
		long src = 0;
		int ghost = 0;
		for (int d = 1; d <= nd; d++) {
			long c = (node / g->sizeProd[d]) % g->size[d];
			int T = g->trueSize[d], G = g->nGhost[d];
			long t = c - G;
			if (t < 0) { t += T; ghost = 1; }
			if (t >= T) { t -= T; ghost = 1; }
			src += (t + G) * g->sizeProd[d];
		}
		if (ghost) v[node] = v[src];
	}
}

OObj *oo_create(OWorld *w, const double *maskTrue) {
	if (w->P != 1) orc_die("object oracle: one subdomain only");
	const OGrid *g = &w->r[0].rho;
	int nd = g->rank - 1;
	if (nd != 3) orc_die("object oracle: 3-D only (object.c)");
	OObj *o = calloc(1, sizeof(*o));
	o->nNodes = g->sizeProd[g->rank];
	o->mask = calloc(o->nNodes, sizeof(double));
	/* maskTrue is [z][y][x] over the true nodes */
	long k = 0;
	for (int z = 0; z < g->trueSize[3]; z++)
		for (int y = 0; y < g->trueSize[2]; y++)
			for (int x = 0; x < g->trueSize[1]; x++) {
				long node = (x + g->nGhost[1]) * g->sizeProd[1] + (y + g->nGhost[2]) * g->sizeProd[2] +
				            (z + g->nGhost[3]) * g->sizeProd[3];
				o->mask[node] = maskTrue[k++];
			}
	fill_ghosts(g, o->mask);
	/* oFillLookupTables: highest id, interior nodes per object */
	int nObj = 0;
	for (long i = 0; i < o->nNodes; i++)
		if (o->mask[i] > nObj) nObj = (int)(o->mask[i] + 0.5);
	o->nObjects = nObj;
	o->interiorOff = calloc(nObj + 1, sizeof(long));
	o->surfaceOff = calloc(nObj + 1, sizeof(long));
	o->objOfNode = calloc(o->nNodes, sizeof(int));
	for (long i = 0; i < o->nNodes; i++)
		if (o->mask[i] > 0.5 && !is_ghost(g, i)) o->interiorOff[(int)(o->mask[i] + 0.5)]++;
	for (int a = 0; a < nObj; a++) o->interiorOff[a + 1] += o->interiorOff[a];
	o->interior = calloc(o->interiorOff[nObj] + 1, sizeof(long));
	long *idx = calloc(nObj + 1, sizeof(long));
	for (int a = 0; a < nObj; a++) idx[a] = o->interiorOff[a];
	for (long i = 0; i < o->nNodes; i++)
		if (o->mask[i] > 0.5 && !is_ghost(g, i)) {
			int a = (int)(o->mask[i] + 0.5);
			o->interior[idx[a - 1]++] = i;
			o->objOfNode[i] = a;
		}
	/* oFindObjectSurfaceNodes: a true node whose 8 surrounding cells'
	 * lower nodes (offsets {0,-1}^3) hold between 1 and 7 nodes of object a */
	const long sx = g->sizeProd[1], sy = g->sizeProd[2], sz = g->sizeProd[3];
	const long nb[8] = {0, -sz, -sx, -sx - sz, -sy, -sy - sz, -sy - sx, -sy - sx - sz};
	for (int pass = 0; pass < 2; pass++) {
		if (pass == 1) {
			for (int a = 0; a < nObj; a++) o->surfaceOff[a + 1] += o->surfaceOff[a];
			o->surface = calloc(o->surfaceOff[nObj] + 1, sizeof(long));
			for (int a = 0; a < nObj; a++) idx[a] = o->surfaceOff[a];
		}
		for (int a = 0; a < nObj; a++)
			for (long b = 0; b < o->nNodes; b++) {
				if (is_ghost(g, b)) continue;
				int d = 0;
				for (int q = 0; q < 8; q++) {
					double v = o->mask[b + nb[q]];
					if (v > a + 0.5 && v < a + 1.5) d++;
				}
				if (d > 0 && d < 8) {
					if (pass == 0) o->surfaceOff[a + 1]++;
					else o->surface[idx[a]++] = b;
				}
			}
	}
	free(idx);
	og_alloc(&o->rhoObj, w->ini, 1);
	og_zero(&o->rhoObj);
	o->collected = calloc(nObj + 1, sizeof(double));
	return o;
}

void oo_free(OObj *o) {
	if (!o) return;
	free(o->mask);
	free(o->objOfNode);
	free(o->interior);
	free(o->interiorOff);
	free(o->surface);
	free(o->surfaceOff);
	free(o->capInv);
	free(o->capOff);
	free(o->capSum);
	free(o->collected);
	og_free(&o->rhoObj);
	free(o);
}

/* Gauss-Jordan inverse with partial pivoting (row-major n x n, in place
 * into inv); the reference uses GSL's LU decomposition + inverse */
static void invert(double *A, double *inv, long n) {
	for (long i = 0; i < n; i++)
		for (long j = 0; j < n; j++) inv[i * n + j] = i == j;
	for (long c = 0; c < n; c++) {
		long p = c;
		for (long r = c + 1; r < n; r++)
			if (fabs(A[r * n + c]) > fabs(A[p * n + c])) p = r;
		if (A[p * n + c] == 0.0) orc_die("capacitance matrix is singular");
		if (p != c)
			for (long j = 0; j < n; j++) {
				double t = A[c * n + j]; A[c * n + j] = A[p * n + j]; A[p * n + j] = t;
				t = inv[c * n + j]; inv[c * n + j] = inv[p * n + j]; inv[p * n + j] = t;
			}
		double d = 1.0 / A[c * n + c];
		for (long j = 0; j < n; j++) { A[c * n + j] *= d; inv[c * n + j] *= d; }
		for (long r = 0; r < n; r++) {
			if (r == c) continue;
			double f = A[r * n + c];
			if (f == 0.0) continue;
			for (long j = 0; j < n; j++) { A[r * n + j] -= f * A[c * n + j]; inv[r * n + j] -= f * inv[c * n + j]; }
		}
	}
}

void oo_capacitance(OObj *o, OWorld *w) {
	OGrid *rho = &w->r[0].rho, *phi = &w->r[0].phi;
	long N = rho->sizeProd[rho->rank];
	double *saveRho = malloc(N * sizeof(double)), *savePhi = malloc(N * sizeof(double));
	memcpy(saveRho, rho->val, N * sizeof(double));
	memcpy(savePhi, phi->val, N * sizeof(double));
	o->capOff = calloc(o->nObjects + 1, sizeof(long));
	for (int a = 0; a < o->nObjects; a++) {
		long n = o->surfaceOff[a + 1] - o->surfaceOff[a];
		o->capOff[a + 1] = o->capOff[a] + n * n;
	}
	o->capInv = calloc(o->capOff[o->nObjects] + 1, sizeof(double));
	o->capSum = calloc(o->nObjects, sizeof(double));
	og_zero(phi);
	for (int a = 0; a < o->nObjects; a++) {
		long n = o->surfaceOff[a + 1] - o->surfaceOff[a];
		const long *sf = o->surface + o->surfaceOff[a];
		double *P = calloc(n * n, sizeof(double));
		for (long i = 0; i < n; i++) {
			og_zero(rho);
			rho->val[sf[i]] = 1.0;
			/* the run's multigrid, as the device (pinc_obj_capacitance):
			 * native mode when configured, with the warm start */
			if (w->native) ow_native_solve(w);
			else ow_mg_solve(w);
			for (long k = 0; k < n; k++) P[k * n + i] = phi->val[sf[k]];
		}
		invert(P, o->capInv + o->capOff[a], n);
		double s = 0;
		for (long l = 0; l < n * n; l++) s += o->capInv[o->capOff[a] + l];
		o->capSum[a] = 1.0 / s;
		free(P);
	}
	memcpy(rho->val, saveRho, N * sizeof(double));
	memcpy(phi->val, savePhi, N * sizeof(double));
	free(saveRho);
	free(savePhi);
	o->haveCap = 1;
}

void oo_apply(OObj *o, OWorld *w, double *phiC) {
	OGrid *rho = &w->r[0].rho;
	const OGrid *phi = &w->r[0].phi;
	for (int a = 0; a < o->nObjects; a++) {
		long n = o->surfaceOff[a + 1] - o->surfaceOff[a];
		const long *sf = o->surface + o->surfaceOff[a];
		const double *M = o->capInv + o->capOff[a];
		if (n <= 0) continue;
		/* eq. 7: phi_c = sum_ij M[j][i] phi_j / sum M (object.c:327-333) */
		double pc = 0;
		for (long i = 0; i < n; i++)
			for (long j = 0; j < n; j++) pc += M[n * j + i] * phi->val[sf[j]];
		pc *= o->capSum[a];
		if (phiC) phiC[a] = pc;
		double *dphi = malloc(n * sizeof(double)), *corr = calloc(n, sizeof(double));
		for (long j = 0; j < n; j++) dphi[j] = pc - phi->val[sf[j]];
		/* eq. 5: rhoCorr_i = sum_j M[j][i] dphi_j (object.c:349-354) */
		for (long i = 0; i < n; i++)
			for (long j = 0; j < n; j++) corr[i] += M[n * j + i] * dphi[j];
		for (long j = 0; j < n; j++) rho->val[sf[j]] += corr[j];
		free(dphi);
		free(corr);
	}
}

/* particles whose cell's lower node is inside an object are removed and
 * their charge counted; the count is spread evenly over the object's
 * surface nodes of rhoObj (object.c:460-515, defects corrected above) */
void oo_collect(OObj *o, OWorld *w) {
	OPop *p = &w->r[0].pop;
	const OGrid *g = &o->rhoObj;
	int nd = p->nDims;
	double *cnt = calloc(o->nObjects + 1, sizeof(double));
	for (int s = 0; s < p->nSpecies; s++) {
		for (long i = p->iStart[s]; i < p->iStop[s];) {
			const double *x = p->pos + i * nd;
			long node = (long)(int)x[0] * g->sizeProd[1] + (long)(int)x[1] * g->sizeProd[2] +
			            (long)(int)x[2] * g->sizeProd[3];
			int a = (node >= 0 && node < o->nNodes) ? o->objOfNode[node] : 0;
			if (a) {
				cnt[a - 1] += p->charge[s];
				long last = p->iStop[s] - 1;
				for (int d = 0; d < nd; d++) {
					p->pos[i * nd + d] = p->pos[last * nd + d];
					p->vel[i * nd + d] = p->vel[last * nd + d];
				}
				if (p->id) p->id[i] = p->id[last];
				p->iStop[s]--;
				continue; /* re-test the particle moved into slot i */
			}
			i++;
		}
	}
	for (int a = 0; a < o->nObjects; a++) {
		long n = o->refDivisor ? o->surfaceOff[a + 1] : o->surfaceOff[a + 1] - o->surfaceOff[a];
		double inv = 1.0 / (double)n;
		o->collected[a] += cnt[a];
		for (long b = o->surfaceOff[a]; b < o->surfaceOff[a + 1]; b++) o->rhoObj.val[o->surface[b]] += cnt[a] * inv;
	}
	free(cnt);
}

/* object.c's own divisor, 1/lookupSurfaceOffset[a+1] (the defect named in
 * the header), for the test that pins the corrected one */
void oo_set_reference_divisor(OObj *o, int on) { o->refDivisor = on; }

/* ctypes accessors */
int oo_nobjects(const OObj *o) { return o->nObjects; }
long oo_nsurface(const OObj *o, int a) { return o->surfaceOff[a + 1] - o->surfaceOff[a]; }
long oo_ninterior(const OObj *o, int a) { return o->interiorOff[a + 1] - o->interiorOff[a]; }
void oo_surface_nodes(const OObj *o, int a, long *out) {
	memcpy(out, o->surface + o->surfaceOff[a], oo_nsurface(o, a) * sizeof(long));
}
void oo_interior_nodes(const OObj *o, int a, long *out) {
	memcpy(out, o->interior + o->interiorOff[a], oo_ninterior(o, a) * sizeof(long));
}
double oo_collected(const OObj *o, int a) { return o->collected[a]; }
void oo_rho_obj(const OObj *o, double *out) {
	memcpy(out, o->rhoObj.val, o->rhoObj.sizeProd[o->rhoObj.rank] * sizeof(double));
}
const OGrid *oo_rho_obj_grid(const OObj *o) { return &o->rhoObj; }
