/*
 * pinc_obj.c -- immersed objects (object.c, config C5) on the device path,
 * any number of z-slabs, fused or unfused operators, either particle layout
 * (with the tiled one the back-filled slots are deposited individually until
 * the next sort, as after a migration).  With a replicated solve phi is read
 * from its global view; with the sharded multigrid (pinc_mg.c, native mode)
 * each rank reads the surface nodes of its own slab and the surface
 * potentials are summed over the ranks (n doubles, as object.c:163-364 does
 * with MPI_Allreduce/Allgather).  Charge corrections go to the owning slab.
 *
 *   pinc_obj_create       oFillLookupTables (object.c:111-160) and
 *                         oFindObjectSurfaceNodes (object.c:368-458) on the
 *                         object mask.  The mask is a sphere given by
 *                         objects:sphere = cx,cy,cz,r in true-node
 *                         coordinates (an extension: the reference reads an
 *                         HDF5 /Object grid, object.c:727-756)
 *   pinc_obj_capacitance  oComputeCapacitanceMatrix (object.c:163-298): one
 *                         device solve per surface node with a unit charge
 *                         there; the inverse (host Gauss-Jordan, GSL's LU in
 *                         the reference) goes to the device.  It uses the
 *                         run's Poisson solver: multigrid as the reference
 *                         (which builds one for it, object.c:176-178) or,
 *                         an extension with parity unpinned, the spectral
 *                         one (exact discrete response)
 *   pinc_obj_collect      oCollectObjectCharge (object.c:460-515): flag kernel
 *                         + the emigrant back-fill (pinc_hip_extract) removes
 *                         the particles; their charge is spread over the
 *                         surface nodes of rhoObj.  With the fused push the
 *                         test rides in k_push (pinc_obj_attach) and the flag
 *                         kernel only sees the immigrants
 *   pinc_obj_add_rho      gAddTo(rho, rhoObj) (main.c:230)
 *   pinc_obj_apply        oApplyCapacitanceMatrix (object.c:301-366)
 *
 * The checker is the object restatement under oracle/,
 * with the same five corrections of reference defects, named in its header:
 *   1. pCut gets the particle, not the node index (object.c:499);
 *   2. the particle swapped into a removed one's slot is re-tested;
 *   3. the unit charge is reset at the object's own surface node
 *      (object.c:243);
 *   4. collected charge is spread with 1/(object a's surface nodes), not
 *      object.c:476-478's 1/lookupSurfaceOffset[a+1] (cumulative: objects
 *      after the first lose charge; tests/test_oracle_objects.py pins both);
 *   5. with several ranks an object's count is summed over the ranks and
 *      spread over all of its surface nodes (the reference spreads each
 *      rank's count over that rank's surface nodes, no reduction: the same
 *      for an object inside one subdomain).
 * Device parity: tests/test_gpu_objects.py.
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>

void pinc_pop_grow_ws(Population *pop, int s, long n);

struct PincObj {
	int nObj;            /* objects: mask values 1..nObj */
	long nSurf;          /* surface nodes of all objects, grouped by object */
	long *surfOff;       /* nObj+1: object a owns surface entries [surfOff[a], surfOff[a+1]) */
	long *surfNode;      /* host: global node index x + T0*(y + T1*z) */
	long *dSurf;         /* device: this rank's slab-storage index of each surface
	                        node, -1 where another rank owns it */
	long *dSurfG;        /* device: index of each surface node in the global
	                        periodic grid the solver works on (phi global view) */
	unsigned char *dInside; /* device: object id per local padded node (0: none) */
	int *dCount;         /* device: particles flagged per object (one species) */
	long nNodes, sy, sz;
	double *dM;          /* device: per object the inverse response matrix, row-major */
	long *capOff;        /* nObj+1 offsets into dM */
	double *wRow;        /* host: sum_i M[j][i] per surface entry j (eq. 7) */
	double *capSum;      /* per object: 1 / sum M */
	double *dPhiS;       /* device: phi at the surface nodes */
	double *rhoObjVal;   /* per object: rhoObj at each of its surface nodes */
	double *collected;   /* per object */
	int haveCap;
	int green;           /* objects:capacitance = green: columns by translation */
	int *dPushCount;     /* device: per species and object, particles the fused push collected */
	int bbLo[3], bbHi[3]; /* bounding box of this rank's interior nodes (padded coordinates) */
	PincDevPop *pop;     /* population attached for the fused collection */
	int T[3];
	/* main.c's order (oAlloc, oOpenH5, oReadH5): the tables are built when
	 * oReadH5 reads the mask named by oOpenH5 */
	int pending;
	int optional;        /* objects:optional = 1 / PINC_OBJ_OPTIONAL=1: no mask file = no objects */
	pinc_geom_t geom;
	char *h5path;
};

static void invert(double *A, double *inv, long n) {
	for (long i = 0; i < n; i++)
		for (long j = 0; j < n; j++) inv[i * n + j] = i == j;
	for (long c = 0; c < n; c++) {
		long p = c;
		for (long r = c + 1; r < n; r++)
			if (fabs(A[r * n + c]) > fabs(A[p * n + c])) p = r;
		if (A[p * n + c] == 0.0) msg(ERROR, "capacitance matrix is singular");
		if (p != c)
			for (long j = 0; j < n; j++) {
				double t = A[c * n + j];
				A[c * n + j] = A[p * n + j];
				A[p * n + j] = t;
				t = inv[c * n + j];
				inv[c * n + j] = inv[p * n + j];
				inv[p * n + j] = t;
			}
		double d = 1.0 / A[c * n + c];
		for (long j = 0; j < n; j++) {
			A[c * n + j] *= d;
			inv[c * n + j] *= d;
		}
		for (long r = 0; r < n; r++) {
			if (r == c) continue;
			double f = A[r * n + c];
			if (f == 0.0) continue;
			for (long j = 0; j < n; j++) {
				A[r * n + j] -= f * A[c * n + j];
				inv[r * n + j] -= f * inv[c * n + j];
			}
		}
	}
}

/* object mask over the true nodes, [z][y][x]: objects:sphere = cx,cy,cz,r
 * (generated) or objects:file = an .h5 file with the reference's /Object
 * dataset [nz, ny, nx, 1] (oReadH5, object.c:727-756) */
static double *read_mask(const dictionary *ini, const int T[3]) {
	long nTrue = (long)T[0] * T[1] * T[2];
	double *mk = calloc(nTrue, sizeof(double));
	if (iniHas(ini, "objects:file")) {
		char *f = iniGetStr(ini, "objects:file");
		long n = pinc_h5_read(f, "/Object", 0, mk, nTrue);
		if (n != nTrue) msg(ERROR, "objects:file=%s: /Object must hold %ld values (got %ld)", f, nTrue, n);
		free(f);
		return mk;
	}
	double *sp = iniGetDoubleArr(ini, "objects:sphere", 4);
	long k = 0;
	for (int z = 0; z < T[2]; z++)
		for (int y = 0; y < T[1]; y++)
			for (int x = 0; x < T[0]; x++, k++) {
				double r2 = (x - sp[0]) * (x - sp[0]) + (y - sp[1]) * (y - sp[1]) + (z - sp[2]) * (z - sp[2]);
				mk[k] = r2 <= sp[3] * sp[3];
			}
	free(sp);
	return mk;
}

static int capacitance_green(const dictionary *ini) {
	int green = 0;
	if (iniHas(ini, "objects:capacitance")) {
		char *c = iniGetStr(ini, "objects:capacitance");
		if (!strcmp(c, "green")) green = 1;
		else if (strcmp(c, "solve")) msg(ERROR, "objects:capacitance=%s (solve or green)", c);
		free(c);
	}
	return green;
}

/* the lookup tables of a mask over the true nodes (mk, [z][y][x] object
 * ids, consumed); an all-zero mask gives an object set with nObj = 0 */
static PincObj *obj_from_mask(double *mk, const pinc_geom_t *g, int green) {
	if (g->nd != 3) msg(ERROR, "objects are 3-D (object.c)");
	PincObj *o = calloc(1, sizeof(*o));
	const int T[3] = {g->T[0], g->T[1], g->T[2]};
	/* this rank's padded nodes: z covers its slab [off, off+nloc) */
	int S[3] = {T[0] + 2, T[1] + 2, g->nloc + 2};
	o->sy = S[0];
	o->sz = (long)S[0] * S[1];
	o->nNodes = o->sz * S[2];
	o->geom = *g;
	/* object ids (oFillLookupTables, object.c:117-121: the highest value is
	 * the object count) */
	int nObj = 0;
	for (long k = 0; k < (long)T[0] * T[1] * T[2]; k++)
		if (mk[k] > nObj) nObj = (int)(mk[k] + 0.5);
	if (nObj > 255) msg(ERROR, "objects: at most 255 objects");
	o->nObj = nObj;
	for (int d = 0; d < 3; d++) o->T[d] = T[d];
	o->green = green;
	if (nObj == 0) {
		free(mk);
		o->haveCap = 1;
		return o;
	}
#define ID(x, y, z) ((int)(mk[((x) + T[0]) % T[0] + (long)T[0] * (((y) + T[1]) % T[1] + (long)T[1] * (((z) + T[2]) % T[2]))] + 0.5))
	/* interior bytes of the local padded nodes (ghosts excluded, as the
	 * reference's lookup skips ghost nodes) */
	unsigned char *inside = calloc(o->nNodes, 1);
	for (long node = 0; node < o->nNodes; node++) {
		int c[3] = {(int)(node % S[0]), (int)((node / o->sy) % S[1]), (int)(node / o->sz)};
		if (c[0] < 1 || c[0] > T[0] || c[1] < 1 || c[1] > T[1] || c[2] < 1 || c[2] > g->nloc) continue;
		int id = ID(c[0] - 1, c[1] - 1, g->off + c[2] - 1);
		inside[node] = (unsigned char)(id > 0 ? id : 0);
	}
	for (int d = 0; d < 3; d++) {
		o->bbLo[d] = 1 << 30;
		o->bbHi[d] = -1;
	}
	for (long node = 0; node < o->nNodes; node++) {
		if (!inside[node]) continue;
		int c[3] = {(int)(node % S[0]), (int)((node / o->sy) % S[1]), (int)(node / o->sz)};
		for (int d = 0; d < 3; d++) {
			if (c[d] < o->bbLo[d]) o->bbLo[d] = c[d];
			if (c[d] > o->bbHi[d]) o->bbHi[d] = c[d];
		}
	}
	if (o->bbHi[0] < 0)
		for (int d = 0; d < 3; d++) { /* no object node in this slab: empty box (hi < lo) */
			o->bbLo[d] = 0;
			o->bbHi[d] = -1;
		}
	/* surface (object.c:368-458): global true nodes with 1..7 of the 8
	 * nodes at offsets {0,-1}^3 in the object, in global z,y,x order (for
	 * z-slabs the reference's rank-then-local order) */
	/* the lists grow geometrically (a surface is a thin shell: sizing them
	 * by the grid would hold GBs at 256^3 with several objects) */
	long nMax = 4096;
	long *dIdx = malloc(nMax * sizeof(long)), *gIdx = malloc(nMax * sizeof(long));
	o->surfNode = malloc(nMax * sizeof(long));
	o->surfOff = calloc(nObj + 1, sizeof(long));
	long ps = (long)T[0] * T[1];
	for (int a = 1; a <= nObj; a++) {
	for (int z = 0; z < T[2]; z++)
		for (int y = 0; y < T[1]; y++)
			for (int x = 0; x < T[0]; x++) {
				int d = 0;
				for (int q = 0; q < 8; q++) d += ID(x - (q & 1), y - ((q >> 1) & 1), z - (q >> 2)) == a;
				if (d > 0 && d < 8) {
					if (o->nSurf == nMax) {
						nMax *= 2;
						dIdx = realloc(dIdx, nMax * sizeof(long));
						gIdx = realloc(gIdx, nMax * sizeof(long));
						o->surfNode = realloc(o->surfNode, nMax * sizeof(long));
						if (!dIdx || !gIdx || !o->surfNode) msg(ERROR, "objects: out of host memory");
					}
					o->surfNode[o->nSurf] = x + (long)T[0] * (y + (long)T[1] * z);
					gIdx[o->nSurf] = (long)z * ps + (long)y * T[0] + x;
					int zl = z - g->off;
					dIdx[o->nSurf] = (zl >= 0 && zl < g->nloc) ? (long)(zl + 1) * ps + (long)y * T[0] + x : -1;
					o->nSurf++;
				}
			}
		o->surfOff[a] = o->nSurf;
	}
#undef ID
	free(mk);
	if (!o->nSurf) msg(ERROR, "objects: the mask has no surface nodes");
	o->surfNode = realloc(o->surfNode, o->nSurf * sizeof(long));
	pinc_check(pinc_hip_malloc((void **)&o->dInside, o->nNodes), "objects");
	pinc_check(pinc_hip_h2d(o->dInside, inside, o->nNodes, g_pinc.stream), "objects");
	pinc_check(pinc_hip_malloc((void **)&o->dSurf, o->nSurf * sizeof(long)), "objects");
	pinc_check(pinc_hip_h2d(o->dSurf, dIdx, o->nSurf * sizeof(long), g_pinc.stream), "objects");
	pinc_check(pinc_hip_malloc((void **)&o->dSurfG, o->nSurf * sizeof(long)), "objects");
	pinc_check(pinc_hip_h2d(o->dSurfG, gIdx, o->nSurf * sizeof(long), g_pinc.stream), "objects");
	pinc_check(pinc_hip_malloc((void **)&o->dPhiS, o->nSurf * sizeof(double)), "objects");
	pinc_check(pinc_hip_malloc((void **)&o->dCount, (nObj + 1) * sizeof(int)), "objects");
	o->capOff = calloc(nObj + 1, sizeof(long));
	o->capSum = calloc(nObj + 1, sizeof(double));
	o->rhoObjVal = calloc(nObj + 1, sizeof(double));
	o->collected = calloc(nObj + 1, sizeof(double));
	for (int a = 0; a < nObj; a++)
		if (o->surfOff[a + 1] == o->surfOff[a]) msg(ERROR, "object %d has no surface nodes", a + 1);
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), "objects");
	free(inside);
	free(dIdx);
	free(gIdx);
	return o;
}

static PincObj *obj_create(const dictionary *ini, const pinc_geom_t *g) {
	if (!iniHas(ini, "objects:sphere") && !iniHas(ini, "objects:file")) return NULL;
	if (g->nd != 3) msg(ERROR, "objects are 3-D (object.c)");
	const int T[3] = {g->T[0], g->T[1], g->T[2]};
	return obj_from_mask(read_mask(ini, T), g, capacitance_green(ini));
}

PincObj *pinc_obj_create(const dictionary *ini, const Grid *rho) {
	if (!iniHas(ini, "objects:sphere") && !iniHas(ini, "objects:file")) return NULL;
	if (rho->rank != 4) msg(ERROR, "objects are 3-D (object.c)");
	return obj_create(ini, &rho->dev->geom);
}

void pinc_obj_free(PincObj *o) {
	if (!o) return;
	if (o->pop) {
		/* a population that outlives the objects tests no object any more */
		o->pop->objInside = NULL;
		o->pop->objCount = NULL;
		o->pop->objOwner = NULL;
	}
	pinc_hip_free(o->dPushCount);
	pinc_hip_free(o->dInside);
	pinc_hip_free(o->dSurf);
	pinc_hip_free(o->dSurfG);
	pinc_hip_free(o->dPhiS);
	pinc_hip_free(o->dM);
	pinc_hip_free(o->dCount);
	free(o->h5path);
	free(o->surfNode);
	free(o->surfOff);
	free(o->capOff);
	free(o->capSum);
	free(o->rhoObjVal);
	free(o->collected);
	free(o->wRow);
	free(o);
}

long pinc_obj_nsurface(const PincObj *o) { return o ? o->nSurf : 0; }
void pinc_obj_forget_pop(PincObj *o) { o->pop = NULL; }
double pinc_obj_collected(const PincObj *o) {
	double t = 0;
	for (int a = 0; o && a < o->nObj; a++) t += o->collected[a];
	return t;
}

/* phi at surface entries [s0, s0 + n) into dst (device): from the solve's
 * global view, or -- sharded solve, no global phi -- from this rank's slab
 * (the solve leaves the owned planes there) with the other ranks' nodes read
 * as zero, summed over the ranks */
static void surface_phi(PincObj *o, const Grid *phi, long s0, long n, double *dst) {
	if (phi->dev->global) {
		pinc_check(pinc_hip_obj_gather(phi->dev->global, o->dSurfG + s0, n, dst, g_pinc.stream), "object gather");
		return;
	}
	pinc_check(pinc_hip_obj_gather(phi->dev->d, o->dSurf + s0, n, dst, g_pinc.stream), "object gather");
	if (g_pinc.nranks > 1) pinc_comm_allreduce_sum(dst, n, "surface phi");
}

/* object.c:163-298: column i = phi at the surface nodes for a unit charge
 * at surface node i (solver warm-started column to column, as the
 * reference's); rho and phi are restored afterwards */
void pinc_obj_capacitance(PincObj *o, Grid *rho, Grid *phi, void *solver,
                          void (*solve)(void *, Grid *, Grid *, const MpiInfo *), const MpiInfo *mpi) {
	if (!o->nObj) return; /* no objects: nothing to solve for */
	long n = o->nSurf, N = rho->dev->n;
	double *saveR = NULL, *saveP = NULL;
	pinc_check(pinc_hip_malloc((void **)&saveR, N * sizeof(double)), "cap save");
	pinc_check(pinc_hip_malloc((void **)&saveP, N * sizeof(double)), "cap save");
	pinc_check(pinc_hip_d2d(saveR, rho->dev->d, N * sizeof(double), g_pinc.stream), "cap save");
	pinc_check(pinc_hip_d2d(saveP, phi->dev->d, N * sizeof(double), g_pinc.stream), "cap save");
	pinc_check(pinc_hip_memset(phi->dev->d, 0, N * sizeof(double), g_pinc.stream), "cap");
	/* several ranks: the solver's global phi is a buffer of its own; the
	 * sharded solve keeps its level 0 in the extended slab */
	double *saveG = NULL, *saveE = NULL;
	long NG = (long)phi->dev->geom.T[0] * phi->dev->geom.T[1] * phi->dev->geom.T[2];
	long NE = phi->dev->ext && phi->dev->ext != phi->dev->d ? (long)phi->dev->extPlanes * phi->dev->planeSize : 0;
	if (phi->dev->ownsGlobal) {
		pinc_check(pinc_hip_malloc((void **)&saveG, NG * sizeof(double)), "cap save");
		pinc_check(pinc_hip_d2d(saveG, phi->dev->global, NG * sizeof(double), g_pinc.stream), "cap save");
		pinc_check(pinc_hip_memset(phi->dev->global, 0, NG * sizeof(double), g_pinc.stream), "cap");
	}
	if (NE) {
		pinc_check(pinc_hip_malloc((void **)&saveE, NE * sizeof(double)), "cap save");
		pinc_check(pinc_hip_d2d(saveE, phi->dev->ext, NE * sizeof(double), g_pinc.stream), "cap save");
		pinc_check(pinc_hip_memset(phi->dev->ext, 0, NE * sizeof(double), g_pinc.stream), "cap");
	}
	double *col = malloc(n * sizeof(double));
	for (int a = 0; a < o->nObj; a++) {
		long na = o->surfOff[a + 1] - o->surfOff[a];
		o->capOff[a + 1] = o->capOff[a] + na * na;
	}
	/* a second call (oComputeCapacitanceMatrix again) replaces the matrix */
	pinc_hip_free(o->dM);
	o->dM = NULL;
	free(o->wRow);
	pinc_check(pinc_hip_malloc((void **)&o->dM, o->capOff[o->nObj] * sizeof(double)), "cap matrix");
	o->wRow = calloc(n, sizeof(double));
	/* objects:capacitance = green (extension): the periodic, neutralised
	 * problem is translation invariant, so the response at node k to a unit
	 * charge at node i is G(r_k - r_i) for the response G to a unit charge
	 * at the origin: one solve instead of one per surface node.  Equal to
	 * the reference's columns to the solver tolerance. */
	double *G = NULL;
	const long TX = o->T[0], TY = o->T[1], TZ = o->T[2];
	if (o->green) {
		long NG = TX * TY * TZ;
		G = malloc(NG * sizeof(double));
		pinc_check(pinc_hip_memset(rho->dev->d, 0, N * sizeof(double), g_pinc.stream), "cap");
		if (phi->dev->geom.off == 0) {
			long i0 = rho->dev->planeSize; /* global (0,0,0) in the slab of rank 0 */
			double one = 1.0;
			pinc_check(pinc_hip_h2d(rho->dev->d + i0, &one, sizeof(double), g_pinc.stream), "cap unit charge");
		}
		solve(solver, rho, phi, mpi);
		if (phi->dev->global) {
			pinc_check(pinc_hip_d2h(G, phi->dev->global, NG * sizeof(double), g_pinc.stream), "cap green");
		} else {
			/* sharded solve: the response's slabs gathered once (set-up only) */
			long ps = phi->dev->planeSize, nl = phi->dev->geom.nloc;
			double *dG = NULL;
			pinc_check(pinc_hip_malloc((void **)&dG, NG * sizeof(double)), "cap green");
			if (g_pinc.nranks > 1) pinc_comm_allgather(phi->dev->d + ps, dG, ps * nl, "cap green gather");
			else pinc_check(pinc_hip_d2d(dG, phi->dev->d + ps, NG * sizeof(double), g_pinc.stream), "cap green");
			pinc_check(pinc_hip_d2h(G, dG, NG * sizeof(double), g_pinc.stream), "cap green");
			pinc_hip_free(dG);
		}
	}
	for (int a = 0; a < o->nObj; a++) {
		long s0 = o->surfOff[a], na = o->surfOff[a + 1] - s0;
		double *P = malloc(na * na * sizeof(double)), *M = malloc(na * na * sizeof(double));
		for (long i = 0; i < na && G; i++) {
			long ni = o->surfNode[s0 + i];
			long xi = ni % TX, yi = (ni / TX) % TY, zi = ni / (TX * TY);
			for (long k = 0; k < na; k++) {
				long nk = o->surfNode[s0 + k];
				long dx = (nk % TX - xi + TX) % TX, dy = ((nk / TX) % TY - yi + TY) % TY,
				     dz = (nk / (TX * TY) - zi + TZ) % TZ;
				P[k * na + i] = G[dx + TX * (dy + TY * dz)];
			}
		}
		for (long i = 0; i < na && !G; i++) {
			pinc_check(pinc_hip_memset(rho->dev->d, 0, N * sizeof(double), g_pinc.stream), "cap");
			pinc_check(pinc_hip_obj_add(rho->dev->d, o->dSurf + s0 + i, 1, 1.0, g_pinc.stream), "cap unit charge");
			solve(solver, rho, phi, mpi);
			surface_phi(o, phi, s0, na, o->dPhiS);
			pinc_check(pinc_hip_d2h(col, o->dPhiS, na * sizeof(double), g_pinc.stream), "cap gather");
			for (long k = 0; k < na; k++) P[k * na + i] = col[k];
		}
		invert(P, M, na);
		double sum = 0;
		for (long j = 0; j < na; j++)
			for (long i = 0; i < na; i++) {
				sum += M[j * na + i];
				o->wRow[s0 + j] += M[j * na + i];
			}
		o->capSum[a] = 1.0 / sum;
		pinc_check(pinc_hip_h2d(o->dM + o->capOff[a], M, na * na * sizeof(double), g_pinc.stream), "cap matrix");
		pinc_check(pinc_hip_stream_sync(g_pinc.stream), "cap matrix");
		free(P);
		free(M);
	}
	pinc_check(pinc_hip_d2d(rho->dev->d, saveR, N * sizeof(double), g_pinc.stream), "cap restore");
	pinc_check(pinc_hip_d2d(phi->dev->d, saveP, N * sizeof(double), g_pinc.stream), "cap restore");
	if (saveG) pinc_check(pinc_hip_d2d(phi->dev->global, saveG, NG * sizeof(double), g_pinc.stream), "cap restore");
	if (saveE) pinc_check(pinc_hip_d2d(phi->dev->ext, saveE, NE * sizeof(double), g_pinc.stream), "cap restore");
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), "cap");
	pinc_hip_free(saveR);
	pinc_hip_free(saveP);
	pinc_hip_free(saveG);
	pinc_hip_free(saveE);
	free(col);
	free(G);
	rho->dev->ghostsValid = phi->dev->ghostsValid = 0;
	o->haveCap = 1;
}

/* Fused push (population:fused = 1): the push tests every particle that
 * stays against the object table (the test of object.c:489-494 on its new
 * position), flags the ones inside PINC_NE_SINK instead of depositing them
 * and counts them per species and object; the next extract removes them
 * with the emigrants' back-fill (k_push, pinc_pusher.c extract). */
void pinc_obj_attach(PincObj *o, Population *pop) {
	PincDevPop *dv = pop->dev;
	if (!o || !o->nObj || !dv->fused) return;
	long n = (long)PINC_MAX_SPECIES * o->nObj;
	pinc_check(pinc_hip_malloc((void **)&o->dPushCount, n * sizeof(int)), "object push counts");
	pinc_check(pinc_hip_memset(o->dPushCount, 0, n * sizeof(int), g_pinc.stream), "object push counts");
	dv->objInside = o->dInside;
	dv->objSy = o->sy;
	dv->objSz = o->sz;
	dv->objNodes = o->nNodes;
	dv->objK = o->nObj;
	dv->objCount = o->dPushCount;
	dv->objOwner = o;
	for (int d = 0; d < 3; d++) {
		dv->objLo[d] = o->bbLo[d];
		dv->objHi[d] = o->bbHi[d];
	}
	o->pop = dv;
}

/* object.c:460-515 (corrected): remove the particles whose cell's lower
 * node is interior, with the emigrant back-fill order; their charge goes
 * to rhoObj's surface nodes.  discard: main.c:163-166 (charge dropped).
 * With the fused push (pinc_obj_attach) the particles that stayed were
 * tested by the push and are gone already (their counts are read here);
 * only the particles imported since -- [depEnd, iStop) of each species --
 * go through the flag pass. */
void pinc_obj_collect(PincObj *o, Population *pop, int discard) {
	if (!o->nObj) return; /* an all-zero mask (main.c with no object) */
	pinc_pop_flush_host(pop);
	PincDevPop *dv = pop->dev;
	int K = o->nObj;
	double *cnt = calloc(K + 1, sizeof(double));
	int *hc = calloc(K + 1, sizeof(int));
	if (dv->objInside && dv->objInside != o->dInside)
		msg(ERROR, "objects: the population is attached to another object table");
	const int fusedPath = dv->objInside && !discard;
	if (!fusedPath) {
		/* every live particle is tested below, also those a fused push has
		 * already deposited into rhoS: drop that deposit, so that distr
		 * deposits the survivors afresh (a particle inside would otherwise
		 * count twice, in rhoS and in rhoObj) */
		dv->depValid = dv->depExtracted = 0;
		/* the reference's API (oAlloc + oCollectObjectCharge, main.c:222)
		 * never attaches: from the next push on, the push tests the object */
		if (dv->fused && !discard) pinc_obj_attach(o, pop);
	}
	if (fusedPath) {
		int ns = pop->nSpecies;
		int *pc = malloc((size_t)ns * K * sizeof(int));
		pinc_check(pinc_hip_d2h(pc, dv->objCount, (size_t)ns * K * sizeof(int), g_pinc.stream), "object push counts");
		pinc_check(pinc_hip_memset(dv->objCount, 0, (size_t)ns * K * sizeof(int), g_pinc.stream), "object push counts");
		for (int s = 0; s < ns; s++)
			for (int a = 0; a < K; a++) cnt[a] += pop->charge[s] * (double)pc[s * K + a];
		free(pc);
	}
	for (int s = 0; s < pop->nSpecies; s++) {
		long first = pop->iStart[s];
		if (fusedPath && dv->depValid && dv->depExtracted) first = dv->depEnd[s];
		long n = pop->iStop[s] - first;
		if (n <= 0) continue;
		for (int attempt = 0;; attempt++) {
			pinc_pop_t p = pinc_devpop(pop);
			p.iStart[s] = first;
			pinc_check(pinc_hip_memset(o->dCount, 0, (K + 1) * sizeof(int), g_pinc.stream), "object count");
			pinc_check(pinc_hip_obj_flag(p, s, o->dInside, o->sy, o->sz, o->nNodes, dv->flags,
			                             dv->chunkCount + dv->chunkBase[s], o->dCount, g_pinc.stream),
			           "object flag");
			long nRem = 0;
			long neCount[PINC_NE_CODES];
			int rc = pinc_hip_extract(p, s, dv->flags, dv->chunkCount + dv->chunkBase[s], 13, PINC_NNE, dv->ws[s],
			                          &nRem, neCount, g_pinc.stream);
			if (rc == PINC_ERR_CAPACITY && attempt == 0) {
				pinc_pop_grow_ws(pop, s, nRem);
				continue;
			}
			pinc_check(rc, "object collect");
			/* the flags written over [first, iStop) are the centre again (the
			 * extraction put the collected ones back); an earlier write's
			 * leavers below first would not be */
			if (dv->flagState[s] != PINC_FLAGS_CLEAN) dv->flagState[s] = PINC_FLAGS_UNKNOWN;
			pinc_check(pinc_hip_d2h(hc, o->dCount, K * sizeof(int), g_pinc.stream), "object count");
			pop->iStop[s] -= nRem;
			/* removals reorder the tail: cell counts and sorted prefix */
			if (nRem && dv->sorted) dv->cntValid[s] = 0;
			if (nRem && dv->tiled && dv->cellValid[s] > first - pop->iStart[s]) dv->cellValid[s] = first - pop->iStart[s];
			/* chargeCounter[a] += charge[s] per particle (object.c:497) */
			for (int a = 0; a < K; a++) cnt[a] += pop->charge[s] * (double)hc[a];
			break;
		}
	}
	dv->flagsValid = 0;
	if (g_pinc.nranks > 1 && K > 0) {
		/* every rank collects in its slab; the object's charge is global */
		double *d = PINC_SLOT(120);
		if (K > 64) msg(ERROR, "objects: at most 64 objects with several ranks");
		pinc_check(pinc_hip_h2d(d, cnt, K * sizeof(double), g_pinc.stream), "collect sum");
		pinc_comm_allreduce_sum(d, K, "collect sum");
		pinc_check(pinc_hip_d2h(cnt, d, K * sizeof(double), g_pinc.stream), "collect sum");
	}
	if (!discard)
		/* object.c:508-513: chargeCounter * invNrSurfNod added per surface node */
		for (int a = 0; a < K; a++) {
			o->collected[a] += cnt[a];
			o->rhoObjVal[a] += cnt[a] * (1.0 / (double)(o->surfOff[a + 1] - o->surfOff[a]));
		}
	free(cnt);
	free(hc);
}

/* gAddTo(rho, rhoObj) (main.c:230): rhoObj is rhoObjVal at every surface
 * node and zero elsewhere */
void pinc_obj_add_rho(PincObj *o, Grid *rho) {
	for (int a = 0; a < o->nObj; a++)
		if (o->rhoObjVal[a] != 0.0)
			pinc_check(pinc_hip_obj_add(rho->dev->d, o->dSurf + o->surfOff[a], o->surfOff[a + 1] - o->surfOff[a],
			                            o->rhoObjVal[a], g_pinc.stream),
			           "rho += rhoObj");
}

/* object.c:301-366; returns phi_c */
double pinc_obj_apply(PincObj *o, Grid *rho, const Grid *phi) {
	if (!o->nObj) return 0.0;
	if (!o->haveCap) msg(ERROR, "objects: capacitance matrix not computed");
	long n = o->nSurf;
	/* phi at every object's surface first: the corrections do not change
	 * phi until the next solve (object.c:313-363 loops the objects) */
	surface_phi(o, phi, 0, n, o->dPhiS);
	double *ph = malloc(n * sizeof(double));
	pinc_check(pinc_hip_d2h(ph, o->dPhiS, n * sizeof(double), g_pinc.stream), "object gather");
	double pc = 0;
	for (int a = 0; a < o->nObj; a++) {
		long s0 = o->surfOff[a], na = o->surfOff[a + 1] - s0;
		/* eq. 7 through the row sums of M (summed once at init) */
		pc = 0;
		for (long j = 0; j < na; j++) pc += o->wRow[s0 + j] * ph[s0 + j];
		pc *= o->capSum[a];
		pinc_check(pinc_hip_obj_correct(o->dM + o->capOff[a], o->dPhiS + s0, na, pc, o->dSurf + s0, rho->dev->d,
		                                g_pinc.stream),
		           "object correct");
	}
	free(ph);
	rho->dev->ghostsValid = 0;
	return pc;
}

/* ---------------------------------------------- the reference's API -- */
/* object.h:8-21: Object is this build's PincObj (include/pinc.h) */

/* object.c:671-699.  With objects:sphere / objects:file (extensions) the
 * tables are built here; otherwise the object waits for oOpenH5 + oReadH5,
 * the reference's order (main.c:95,126-127). */
Object *oAlloc(const dictionary *ini) {
	pinc_geom_t g = pinc_geom_current();
	PincObj *o = obj_create(ini, &g);
	if (o) return o;
	o = calloc(1, sizeof(*o));
	o->pending = 1;
	o->optional = (iniHas(ini, "objects:optional") && iniGetInt(ini, "objects:optional")) ||
	              (getenv("PINC_OBJ_OPTIONAL") && atoi(getenv("PINC_OBJ_OPTIONAL")));
	o->geom = g;
	o->green = capacitance_green(ini);
	o->haveCap = 1; /* nothing to solve until a mask arrives */
	return o;
}

void oFree(Object *obj) { pinc_obj_free(obj); }

/* object.c:721-725 -> gOpenH5 -> openH5File (io.c:566-602): the file is
 * <files:output><sep><fName>.grid.h5, sep "_" unless the prefix ends in "/"
 * ("/" if it is "."); only its /Object dataset is read */
void oOpenH5(const dictionary *ini, Object *obj, const MpiInfo *mpiInfo, const Units *units, double denorm,
             const char *fName) {
	(void)mpiInfo;
	(void)units;
	(void)denorm;
	char *pre = iniGetStr(ini, "files:output");
	size_t n = strlen(pre);
	const char *sep = !strcmp(pre, ".") ? "/" : (n > 0 && pre[n - 1] != '/' ? "_" : "");
	free(obj->h5path);
	if (asprintf(&obj->h5path, "%s%s%s.grid.h5", pre, sep, fName) < 0) msg(ERROR, "oOpenH5: out of memory");
	free(pre);
}

/* object.c:727-756: read /Object, then oFillLookupTables and
 * oFindObjectSurfaceNodes.  An object built from the ini (extensions) keeps
 * its tables.  No file at the oOpenH5 path ends the run, as in the
 * reference (its H5Dopen fails); a run without objects must opt in with
 * objects:optional = 1 or PINC_OBJ_OPTIONAL=1 (a mistyped
 * files:output must not run silently without the objects). */
void oReadH5(Object *obj, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	if (!obj->pending) return;
	obj->pending = 0;
	if (!obj->h5path) msg(ERROR, "oReadH5 before oOpenH5");
	FILE *f = fopen(obj->h5path, "rb");
	if (!f) {
		if (!obj->optional)
			msg(ERROR, "oReadH5: no object mask %s (set objects:optional=1 to run without objects)", obj->h5path);
		msg(WARNING, "oReadH5: no %s, the run has no objects (objects:optional)", obj->h5path);
		return;
	}
	fclose(f);
	const int *T = obj->geom.T;
	long nTrue = (long)T[0] * T[1] * T[2];
	double *mk = calloc(nTrue, sizeof(double));
	long got = pinc_h5_read(obj->h5path, "/Object", 0, mk, nTrue);
	if (got != nTrue)
		msg(ERROR, "oReadH5: %s /Object must hold %ld values (grid %dx%dx%d), got %ld", obj->h5path, nTrue, T[0],
		    T[1], T[2], got);
	PincObj *t = obj_from_mask(mk, &obj->geom, obj->green);
	t->h5path = obj->h5path;
	*obj = *t; /* the caller holds obj */
	free(t);
	if (obj->nObj) msg(STATUS, "oReadH5: %d object(s), %ld surface nodes", obj->nObj, obj->nSurf);
}

void oCloseH5(Object *obj) { (void)obj; /* nothing stays open (the read opens and closes) */ }

/* object.c:163-298: the reference allocates its own solver for the columns */
void oComputeCapacitanceMatrix(Object *obj, const dictionary *ini, const MpiInfo *mpiInfo) {
	if (!obj->nObj) return;
	Grid *rho = gAlloc(ini, SCALAR), *phi = gAlloc(ini, SCALAR);
	MultigridSolver *S = mgAllocSolver(ini, rho, phi);
	pinc_obj_capacitance(obj, rho, phi, S, (void (*)(void *, Grid *, Grid *, const MpiInfo *))mgSolve, mpiInfo);
	mgFreeSolver(S);
	gFree(rho);
	gFree(phi);
}

void oApplyCapacitanceMatrix(Grid *rho, const Grid *phi, const Object *obj, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	if (!obj->nObj) return;
	pinc_obj_apply((PincObj *)obj, rho, phi);
}

/* object.c:460-515: the collected charge is added to rhoObj's surface nodes */
void oCollectObjectCharge(Population *pop, Grid *rhoObj, Object *obj, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	double before[256];
	for (int a = 0; a < obj->nObj; a++) before[a] = obj->rhoObjVal[a];
	pinc_obj_collect(obj, pop, 0);
	for (int a = 0; a < obj->nObj; a++) {
		double add = obj->rhoObjVal[a] - before[a];
		if (add != 0.0)
			pinc_check(pinc_hip_obj_add(rhoObj->dev->d, obj->dSurf + obj->surfOff[a],
			                            obj->surfOff[a + 1] - obj->surfOff[a], add, g_pinc.stream),
			           "rhoObj");
	}
}
