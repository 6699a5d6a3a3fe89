/*
 * pinc_grid.c -- Grid and MpiInfo with device twins (host side, C).
 *
 *   gAlloc / gFree          grid.c:413-500 (+ device slab, DESIGN.md "Layout")
 *   gAllocMpi               grid.c:502-545, getSubdomain grid.c:149-176
 *   gCreateNeighborhood     grid.c:1029-1132 (thresholds, emigrant sizes)
 *   gHaloOp                 grid.c:340-406: periodic dims are index wraps on
 *                           the device; the slab dimension is a self-fold
 *                           (one rank) or an RCCL exchange with z+-1
 *   gFinDiff1st             grid.c:226-261
 *   gMul/gZero/gAddTo       grid.c:668-802
 *   gNeutralizeGrid         grid.c:730-779 (+ RCCL allreduce)
 *   gPotEnergy              grid.c:1276-1321
 *   gSyncToHost/ToDevice    reference-layout host mirror <-> device
 * Only the decomposition nSubdomains = (1,..,1,P) is supported on the
 * device (one slab per GPU along the last dimension).
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>

static pinc_geom_t g_geom; /* geometry of this rank (set by gAllocMpi) */
static int g_geomSet = 0;

pinc_geom_t pinc_geom_current(void) {
	if (!g_geomSet) msg(ERROR, "grid geometry used before gAllocMpi");
	return g_geom;
}
void pinc_geom_set(pinc_geom_t g) {
	g_geom = g;
	g_geomSet = 1;
}

MpiInfo *gAllocMpi(const dictionary *ini) {
	pinc_ctx_require();
	int nd = iniGetInt(ini, "grid:nDims");
	int ns = iniGetInt(ini, "population:nSpecies");
	if (nd < 1 || nd > 3) msg(ERROR, "grid:nDims must be 1, 2 or 3");
	if (ns < 1 || ns > PINC_MAX_SPECIES) msg(ERROR, "population:nSpecies must be 1..%d", PINC_MAX_SPECIES);
	int *nsub = iniGetIntArr(ini, "grid:nSubdomains", nd);
	int *ng = iniGetIntArr(ini, "grid:nGhostLayers", 2 * nd);
	int *ts = iniGetIntArr(ini, "grid:trueSize", nd);
	int total = 1;
	for (int d = 0; d < nd; d++) total *= nsub[d];
	if (total != g_pinc.nranks)
		msg(ERROR, "The product of grid:nSubdomains does not match the number of processes");
	for (int d = 0; d < nd - 1; d++)
		if (nsub[d] != 1) msg(ERROR, "MI355X path decomposes the last dimension only (grid:nSubdomains=1,..,1,P)");
	for (int d = 0; d < 2 * nd; d++)
		if (ng[d] != 1) msg(ERROR, "grid:nGhostLayers must be 1 (grid.h:39)");
	MpiInfo *m = calloc(1, sizeof(*m));
	m->mpiRank = g_pinc.rank;
	m->mpiSize = g_pinc.nranks;
	m->nDims = nd;
	m->nSpecies = ns;
	m->subdomain = calloc(nd, sizeof(int));
	m->nSubdomains = nsub;
	m->nSubdomainsProd = calloc(nd + 1, sizeof(int));
	m->offset = calloc(nd, sizeof(int));
	m->posToSubdomain = calloc(nd, sizeof(double));
	m->nSubdomainsProd[0] = 1;
	int r = m->mpiRank;
	for (int d = 0; d < nd; d++) {
		m->nSubdomainsProd[d + 1] = m->nSubdomainsProd[d] * nsub[d];
		m->subdomain[d] = r % nsub[d];
		r /= nsub[d];
		m->offset[d] = m->subdomain[d] * ts[d] - ng[d];
		m->posToSubdomain[d] = (double)1 / ts[d];
	}
	m->comm = g_pinc.comm;
	pinc_geom_t g;
	memset(&g, 0, sizeof(g));
	g.nd = nd;
	for (int d = 0; d < 3; d++) g.T[d] = d < nd ? ts[d] * nsub[d] : 1;
	g.nloc = ts[nd - 1];
	g.off = m->subdomain[nd - 1] * ts[nd - 1];
	g.nranks = nsub[nd - 1];
	pinc_geom_set(g);
	free(ng);
	free(ts);
	return m;
}

void gFreeMpi(MpiInfo *m) {
	if (!m) return;
	gDestroyNeighborhood(m);
	free(m->subdomain);
	free(m->nSubdomains);
	free(m->nSubdomainsProd);
	free(m->offset);
	free(m->posToSubdomain);
	free(m);
}

static PincDevGrid *g_live;          /* allocated grids (pinc_grid_live) */
static unsigned long long g_serial;

int pinc_grid_live(const Grid *g, unsigned long long serial) {
	for (const PincDevGrid *d = g_live; d; d = d->liveNext)
		if (d->serial == serial) return g->dev == d;
	return 0;
}

Grid *gAlloc(const dictionary *ini, int nValues) {
	pinc_geom_t geo = pinc_geom_current();
	int nd = iniGetInt(ini, "grid:nDims");
	int *ts = iniGetIntArr(ini, "grid:trueSize", nd);
	char **bnds = iniGetStrArr(ini, "grid:boundaries", 2 * nd);
	int rank = nd + 1;
	if (nValues == VECTOR) nValues = nd;
	Grid *g = calloc(1, sizeof(*g));
	g->rank = rank;
	g->size = calloc(rank, sizeof(int));
	g->trueSize = calloc(rank, sizeof(int));
	g->nGhostLayers = calloc(2 * rank, sizeof(int));
	g->sizeProd = calloc(rank + 1, sizeof(long));
	g->bnd = calloc(2 * rank, sizeof(bndType));
	g->size[0] = g->trueSize[0] = nValues;
	for (int d = 1; d < rank; d++) {
		g->trueSize[d] = ts[d - 1];
		g->nGhostLayers[d] = g->nGhostLayers[d + rank] = 1;
		g->size[d] = ts[d - 1] + 2;
	}
	g->sizeProd[0] = 1;
	for (int d = 0; d < rank; d++) g->sizeProd[d + 1] = g->sizeProd[d] * g->size[d];
	for (int b = 0, r = 0; r < 2 * rank; r++) {
		if (r % rank == 0) {
			g->bnd[r] = NONE;
			continue;
		}
		if (!strcmp(bnds[b], "PERIODIC")) g->bnd[r] = PERIODIC;
		else if (!strcmp(bnds[b], "DIRICHLET") || !strcmp(bnds[b], "NEUMANN"))
			msg(ERROR, "%s boundaries are not on the MI355X hot path (periodic only)", bnds[b]);
		else msg(ERROR, "%s invalid value for grid:boundaries", bnds[b]);
		b++;
	}
	freeStrArr(bnds);
	free(ts);
	PincDevGrid *dv = calloc(1, sizeof(*dv));
	dv->nValues = nValues;
	dv->geom = geo;
	dv->planeSize = 1;
	for (int d = 0; d < nd - 1; d++) dv->planeSize *= geo.T[d];
	dv->n = dv->planeSize * (geo.nloc + 2) * nValues;
	pinc_check(pinc_hip_malloc((void **)&dv->d, dv->n * sizeof(double)), "gAlloc");
	pinc_check(pinc_hip_memset(dv->d, 0, dv->n * sizeof(double), g_pinc.stream), "gAlloc zero");
	if (g_pinc.nranks > 1) {
		pinc_check(pinc_hip_malloc((void **)&dv->recv[0], dv->planeSize * nValues * sizeof(double)), "halo buf");
		pinc_check(pinc_hip_malloc((void **)&dv->recv[1], dv->planeSize * nValues * sizeof(double)), "halo buf");
	}
	dv->serial = ++g_serial;
	dv->liveNext = g_live;
	g_live = dv;
	g->dev = dv;
	return g;
}

void gFree(Grid *g) {
	if (!g) return;
	if (g->dev) {
		pinc_grid_touch(g); /* a pending sorting push that kicked with it lets go first */
		for (PincDevGrid **l = &g_live; *l; l = &(*l)->liveNext)
			if (*l == g->dev) {
				*l = g->dev->liveNext;
				break;
			}
		pinc_hip_free(g->dev->d);
		if (g->dev->ownsGlobal) pinc_hip_free(g->dev->global);
		pinc_hip_free(g->dev->recv[0]);
		pinc_hip_free(g->dev->recv[1]);
		pinc_hip_free(g->dev->scaled);
		pinc_hip_free(g->dev->scaledAll);
		pinc_hip_free(g->dev->lit);
		free(g->dev);
	}
	free(g->val);
	free(g->size);
	free(g->trueSize);
	free(g->nGhostLayers);
	free(g->sizeProd);
	free(g->bnd);
	free(g);
}

void gSetBndSlices(Grid *grid, MpiInfo *mpiInfo) {
	(void)grid;
	(void)mpiInfo; /* periodic boundaries need no boundary slices (grid.c:608-666) */
}

void gCreateNeighborhood(const dictionary *ini, MpiInfo *m, Grid *grid) {
	int nd = m->nDims, ns = m->nSpecies;
	int nN = pinc_ipow3(nd);
	int center = 0;
	for (int i = 0; i < nd; i++) center += pinc_ipow3(i);
	int nTest = iniGetNElements(ini, "grid:nEmigrantsAlloc");
	if (nTest != nN && nTest != 1 && nTest != nd)
		msg(ERROR, "grid:nEmigrantsAlloc must consist of 1, nDims=%i or 3^nDims=%i elements", nd, nN);
	long *tmp = iniGetLongIntArr(ini, "grid:nEmigrantsAlloc", nTest);
	m->nEmigrantsAlloc = calloc(nN, sizeof(long));
	for (int ne = 0; ne < nN; ne++) {
		if (ne == center) continue;
		if (nTest == 1) m->nEmigrantsAlloc[ne] = tmp[0];
		else if (nTest == nN) m->nEmigrantsAlloc[ne] = tmp[ne];
		else {
			int t = ne, dims = nd;
			for (int d = nd - 1; d >= 0; d--) {
				int pw = pinc_ipow3(d);
				if (t / pw != 1) dims--;
				t %= pw;
			}
			m->nEmigrantsAlloc[ne] = tmp[dims];
		}
	}
	free(tmp);
	double *thr = iniGetDoubleArr(ini, "grid:thresholds", 2 * nd);
	m->thresholds = calloc(3 * nd, sizeof(double));
	for (int i = 0; i < nd; i++) m->thresholds[i] = thr[i];
	for (int i = nd; i < 2 * nd; i++) m->thresholds[i] = (grid->size[i % nd + 1] - 1) - thr[i];
	/* upper bound of pPosAssertInLocalFrame (population.c:316-340) */
	for (int i = 0; i < nd; i++) m->thresholds[2 * nd + i] = grid->size[i + 1] - 1;
	free(thr);
	/* puMove classifies in the same pass, so it needs the thresholds too */
	for (int i = 0; i < 3 * nd; i++) g_pinc.thr[i] = m->thresholds[i];
	g_pinc.thrSet = 1;
	m->nNeighbors = nN;
	m->neighborhoodCenter = center;
	m->nEmigrants = calloc(nN * ns, sizeof(long));
	m->nImmigrants = calloc(nN * ns, sizeof(long));
}

void gDestroyNeighborhood(MpiInfo *m) {
	free(m->nEmigrantsAlloc);
	free(m->nEmigrants);
	free(m->nImmigrants);
	free(m->thresholds);
	m->nEmigrantsAlloc = m->nEmigrants = m->nImmigrants = NULL;
	m->thresholds = NULL;
	m->nNeighbors = 0;
}

/* slice operators: only their identity is used (token semantics) */
void setSlice(const double *slice, Grid *grid, int d, int offset) {
	(void)slice; (void)grid; (void)d; (void)offset;
	msg(ERROR, "setSlice is a halo token on the device path");
}
void addSlice(const double *slice, Grid *grid, int d, int offset) {
	(void)slice; (void)grid; (void)d; (void)offset;
	msg(ERROR, "addSlice is a halo token on the device path");
}

/* Send plane upPlane to the upper slab and plane downPlane to the lower one.
 * recv[0] receives what the lower slab sent up, recv[1] what the upper slab
 * sent down (grid.c:392-402, tags 1 and 0). */
static void exchange_planes(Grid *g, int upPlane, int downPlane) {
	PincDevGrid *dv = g->dev;
	int P = g_pinc.nranks, r = g_pinc.rank;
	int up = (r + 1) % P, dn = (r - 1 + P) % P;
	long ps = dv->planeSize * dv->nValues;
	long bytes = ps * sizeof(double);
	int sp[2] = {up, dn}, rp[2] = {dn, up};
	void *sb[2] = {dv->d + (long)upPlane * ps, dv->d + (long)downPlane * ps};
	void *rb[2] = {dv->recv[0], dv->recv[1]};
	long nb[2] = {bytes, bytes};
	pinc_comm_exchange(2, sp, sb, nb, rp, rb, nb, "halo exchange");
}

/* Refresh the h halo planes on each side of an extended slab (nloc owned
 * planes at [h, h+nloc), planes of ps nodes) from the neighbouring slabs,
 * z-1 below and z+1 above, periodic; on one rank the halo is the slab's own
 * periodic image.  Collective over the ranks. */
void pinc_ext_halo(double *a, long ps, int nloc, int h) {
	long bytes = (long)h * ps * sizeof(double);
	if (g_pinc.nranks == 1) {
		pinc_check(pinc_hip_d2d(a, a + (long)nloc * ps, bytes, g_pinc.stream), "ext halo");
		pinc_check(pinc_hip_d2d(a + (long)(h + nloc) * ps, a + (long)h * ps, bytes, g_pinc.stream), "ext halo");
		return;
	}
	int P = g_pinc.nranks, r = g_pinc.rank;
	int up = (r + 1) % P, dn = (r - 1 + P) % P;
	/* top owned planes [nloc, nloc+h) go up into the upper slab's lower halo,
	 * bottom owned planes [h, 2h) go down into the lower slab's upper halo */
	int sp[2] = {up, dn}, rp[2] = {dn, up};
	void *sb[2] = {a + (long)nloc * ps, a + (long)h * ps};
	void *rb[2] = {a, a + (long)(h + nloc) * ps};
	long nb[2] = {bytes, bytes};
	pinc_comm_exchange(2, sp, sb, nb, rp, rb, nb, "ext halo");
}

void gHaloOp(funPtr sliceOp, Grid *grid, const MpiInfo *mpiInfo, opDirection dir) {
	(void)mpiInfo;
	PincDevGrid *dv = grid->dev;
	pinc_geom_t geo = dv->geom;
	long ps = dv->planeSize * dv->nValues;
	int nl = geo.nloc;
	if (sliceOp == (funPtr)addSlice && dir == FROMHALO) {
		/* main.c:232's second fold of one deposit (main.c:226 was the first) */
		if (dv->depPop && dv->folds == 1 && !geo.literal) pinc_literal_second_fold(dv->depPop, grid, dv->depOrder);
		dv->folds++;
		pinc_grid_touch(grid);
		if (g_pinc.nranks == 1) {
			pinc_check(pinc_hip_fold_self(dv->d, geo, g_pinc.stream), "fold");
		} else {
			/* ghost nloc+1 goes up and lands on the upper rank's plane 1;
			 * ghost 0 goes down and lands on the lower rank's plane nloc */
			exchange_planes(grid, nl + 1, 0);
			pinc_check(pinc_hip_add(dv->d + ps, dv->recv[0], ps, g_pinc.stream), "halo add");
			pinc_check(pinc_hip_add(dv->d + (long)nl * ps, dv->recv[1], ps, g_pinc.stream), "halo add");
		}
		dv->ghostsValid = 0;
		return;
	}
	if (sliceOp == (funPtr)setSlice && dir == TOHALO) {
		if (dv->ghostsValid) return;
		pinc_grid_touch(grid);
		if (dv->global) {
			pinc_check(pinc_hip_slab_from_global(dv->d, dv->global, geo, dv->nValues, g_pinc.stream),
			           "slab from global");
		} else if (g_pinc.nranks == 1) {
			pinc_check(pinc_hip_d2d(dv->d, dv->d + (long)nl * ps, ps * sizeof(double), g_pinc.stream), "halo");
			pinc_check(pinc_hip_d2d(dv->d + (long)(nl + 1) * ps, dv->d + ps, ps * sizeof(double), g_pinc.stream),
			           "halo");
		} else {
			/* true plane nloc goes up into the upper rank's ghost 0, true
			 * plane 1 goes down into the lower rank's ghost nloc+1 */
			exchange_planes(grid, nl, 1);
			pinc_check(pinc_hip_d2d(dv->d, dv->recv[0], ps * sizeof(double), g_pinc.stream), "halo");
			pinc_check(pinc_hip_d2d(dv->d + (long)(nl + 1) * ps, dv->recv[1], ps * sizeof(double), g_pinc.stream),
			           "halo");
		}
		dv->ghostsValid = 1;
		if (dv->ext == dv->d) dv->extStale = 0; /* the slab is the extended view */
		return;
	}
	msg(ERROR, "gHaloOp: unsupported slice operation / direction on the device path");
}

static void fin_diff(const Grid *scalar, Grid *field, double h);

void gFinDiff1st(const Grid *scalar, Grid *field) { fin_diff(scalar, field, 0.5); }

/* gFinDiff1st followed by gMul(field, -1) in one pass, bit for bit the two
 * (the step of regular(): main.c:245-247, where the TOHALO between them
 * commutes with the exact negation) */
void pinc_fin_diff_neg(const Grid *scalar, Grid *field) { fin_diff(scalar, field, -0.5); }

static void fin_diff(const Grid *scalar, Grid *field, double h) {
	pinc_grid_touch(field);
	if (scalar->dev->ext) {
		/* sharded multigrid: the extended slab holds planes off-hz .. of the
		 * potential, every plane E reads exact (pinc_mg.c) */
		PincDevGrid *sv = scalar->dev;
		if (sv->extStale) {
			pinc_ext_halo(sv->ext, sv->planeSize, sv->geom.nloc, sv->extOff);
			sv->extStale = 0;
		}
		pinc_geom_t g = field->dev->geom;
		g.T[g.nd - 1] = scalar->dev->extPlanes;
		g.off = scalar->dev->extOff;
		pinc_check(pinc_hip_efield_scaled(scalar->dev->ext, g, field->dev->d, h, g_pinc.stream), "efield");
		/* a halo of one plane gives E on the true planes only: its ghost
		 * planes then come from the neighbours (TOHALO) */
		field->dev->ghostsValid = sv->extOff >= 2;
		return;
	}
	const double *phi = scalar->dev->global ? scalar->dev->global : scalar->dev->d + scalar->dev->planeSize;
	if (!scalar->dev->global && g_pinc.nranks > 1)
		msg(ERROR, "gFinDiff1st needs the global potential (run the solver first)");
	pinc_check(pinc_hip_efield_scaled(phi, field->dev->geom, field->dev->d, h, g_pinc.stream), "efield");
	field->dev->ghostsValid = 1;
}

void gMul(Grid *grid, double num) {
	pinc_grid_touch(grid);
	pinc_check(pinc_hip_scale(grid->dev->d, grid->dev->n, num, g_pinc.stream), "gMul");
}

void gZero(Grid *grid) {
	pinc_grid_touch(grid);
	pinc_check(pinc_hip_zero(grid->dev->d, grid->dev->n, g_pinc.stream), "gZero");
	grid->dev->ghostsValid = 0;
	grid->dev->depPop = NULL;
}

void gAddTo(Grid *result, Grid *addition) {
	pinc_grid_touch(result);
	pinc_check(pinc_hip_add(result->dev->d, addition->dev->d, result->dev->n, g_pinc.stream), "gAddTo");
}

void gNeutralizeGrid(Grid *grid, const MpiInfo *mpiInfo) {
	(void)mpiInfo;
	PincDevGrid *dv = grid->dev;
	long ps = dv->planeSize * dv->nValues;
	long nTrue = ps * dv->geom.nloc;
	pinc_check(pinc_hip_sum(dv->d + ps, nTrue, g_pinc.dScratch, PINC_SLOT(1), g_pinc.stream), "neutralize sum");
	if (g_pinc.nranks > 1)
		pinc_comm_allreduce_sum(PINC_SLOT(1), 1, "neutralize allreduce");
	double tot = 0;
	pinc_check(pinc_hip_d2h(&tot, PINC_SLOT(1), sizeof(double), g_pinc.stream), "neutralize");
	double avg = tot / ((double)nTrue * g_pinc.nranks);
	pinc_check(pinc_hip_h2d(PINC_SLOT(2), &avg, sizeof(double), g_pinc.stream), "neutralize");
	pinc_check(pinc_hip_sub_dev(dv->d, dv->n, PINC_SLOT(2), g_pinc.stream), "neutralize sub");
}

/* 0.5 * sum over this rank's true nodes of rho*phi (grid.c:1276-1294):
 * the sum into PINC_SLOT(3), read by gPotEnergy (or by the step loop
 * together with the error word, pinc_regular.c) */
void pinc_pot_energy_launch(const Grid *rho, const Grid *phi) {
	const PincDevGrid *r = rho->dev, *p = phi->dev;
	long ps = r->planeSize;
	long n = ps * r->geom.nloc;
	const double *rv = r->global ? r->global + (long)r->geom.off * ps : r->d + ps;
	const double *pv = p->global ? p->global + (long)p->geom.off * ps : p->d + ps;
	if (g_pinc.nranks == 1) {
		rv = r->global ? r->global : r->d + ps;
		pv = p->global ? p->global : p->d + ps;
	}
	pinc_check(pinc_hip_dot(rv, pv, n, g_pinc.dScratch, PINC_SLOT(3), g_pinc.stream), "potential energy");
}

void gPotEnergy(const Grid *rho, const Grid *phi, Population *pop) {
	pinc_pot_energy_launch(rho, phi);
	double e = 0;
	pinc_check(pinc_hip_d2h(&e, PINC_SLOT(3), sizeof(double), g_pinc.stream), "potential energy");
	pop->potEnergy[pop->nSpecies] = 0.5 * e;
}

/* --------------------------------------------------------------- sync -- */
/* reference-layout node (padded coords) -> device slab node */
static long slab_node(const PincDevGrid *dv, const int *c) {
	pinc_geom_t g = dv->geom;
	long idx = 0, stride = 1;
	for (int d = 0; d < g.nd; d++) {
		int s;
		long ext;
		if (d == g.nd - 1) {
			s = c[d];
			ext = g.nloc + 2;
		} else {
			s = c[d] - 1;
			if (s < 0) s += g.T[d];
			if (s >= g.T[d]) s -= g.T[d];
			ext = g.T[d];
		}
		idx += s * stride;
		stride *= ext;
	}
	return idx;
}

void gSyncToHost(Grid *grid) {
	PincDevGrid *dv = grid->dev;
	/* the potential's truth is the solver's global view: bring the slab (and
	 * its ghost planes) up to date first.  rho's slab is its own truth, ghost
	 * planes included: a gWriteH5 between main.c's two folds (main.c:226-232)
	 * must not replace the ghost deposits with periodic images */
	if (dv->global && dv->globalIsTruth) gHaloOp((funPtr)setSlice, grid, NULL, TOHALO);
	int rank = grid->rank;
	long total = grid->sizeProd[rank];
	if (!grid->val) grid->val = calloc(total, sizeof(double));
	double *tmp = malloc(dv->n * sizeof(double));
	pinc_check(pinc_hip_d2h(tmp, dv->d, dv->n * sizeof(double), g_pinc.stream), "gSyncToHost");
	int nv = dv->nValues, nd = rank - 1;
	int c[3] = {0, 0, 0};
	for (long node = 0; node < total / nv; node++) {
		long r = node;
		for (int d = 0; d < nd; d++) {
			c[d] = (int)(r % grid->size[d + 1]);
			r /= grid->size[d + 1];
		}
		long s = slab_node(dv, c);
		for (int v = 0; v < nv; v++) grid->val[node * nv + v] = tmp[s * nv + v];
	}
	free(tmp);
}

void gSyncToDevice(Grid *grid) {
	PincDevGrid *dv = grid->dev;
	pinc_grid_touch(grid);
	if (!grid->val) msg(ERROR, "gSyncToDevice without host values");
	int rank = grid->rank, nd = rank - 1, nv = dv->nValues;
	double *tmp = malloc(dv->n * sizeof(double));
	pinc_check(pinc_hip_d2h(tmp, dv->d, dv->n * sizeof(double), g_pinc.stream), "gSyncToDevice");
	long total = grid->sizeProd[rank];
	int c[3] = {0, 0, 0};
	for (long node = 0; node < total / nv; node++) {
		long r = node;
		int interior = 1;
		for (int d = 0; d < nd; d++) {
			c[d] = (int)(r % grid->size[d + 1]);
			r /= grid->size[d + 1];
			if (d < nd - 1 && (c[d] == 0 || c[d] == grid->size[d + 1] - 1)) interior = 0;
		}
		if (!interior) continue; /* non-slab ghosts are periodic images on the device */
		long s = slab_node(dv, c);
		for (int v = 0; v < nv; v++) tmp[s * nv + v] = grid->val[node * nv + v];
	}
	pinc_check(pinc_hip_h2d(dv->d, tmp, dv->n * sizeof(double), g_pinc.stream), "gSyncToDevice");
	free(tmp);
	if (dv->ext) {
		/* sharded multigrid: the owned planes of the extended slab (its halo
		 * is refreshed before every smoothing chunk); distributed spectral:
		 * the slab itself */
		long ps = dv->planeSize;
		if (dv->ext != dv->d)
			pinc_check(pinc_hip_d2d(dv->ext + (long)dv->extOff * ps, dv->d + ps, ps * dv->geom.nloc * sizeof(double),
			                        g_pinc.stream), "gSyncToDevice ext");
		dv->ghostsValid = 0;
		dv->extStale = 1;
		return;
	}
	if (dv->global && dv->ownsGlobal) {
		long ps = dv->planeSize * nv;
		pinc_check(pinc_hip_d2d(dv->global + (long)dv->geom.off * ps, dv->d + ps,
		                        ps * dv->geom.nloc * sizeof(double), g_pinc.stream), "gSyncToDevice global");
	}
	dv->ghostsValid = 0;
}
