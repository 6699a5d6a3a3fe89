/*
 * pinc_pop.c -- Population with its device twin (host side, C).
 *
 *   pAlloc / pFree         population.c:42-108 (+ SoA device arrays)
 *   pPosLattice            population.c:172-240   (host mirror)
 *   pPosPerturb            population.c:242-276   (host mirror)
 *   pVelZero / pVelMaxwell population.c:367-428   (counter RNG; GSL absent)
 *   pToLocal/GlobalFrame   population.c:727-763
 *   pSumKinEnergy          population.c:700-709
 *   pInitDevice            the same initial state generated on the GPU
 *   pSyncToHost/ToDevice   AoS host mirror <-> SoA device arrays
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>

static long *g_hostIds = NULL; /* lattice index of each host particle */

static void ws_alloc(pinc_extract_ws_t *ws, long cap) {
	memset(ws, 0, sizeof(*ws));
	ws->cap = cap;
	pinc_check(pinc_hip_malloc((void **)&ws->tail, (cap + 2) * sizeof(int)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->holes, (cap + 2) * sizeof(int)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->order, (cap + 2) * sizeof(int)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->blockHist, (PINC_NE_CODES * (cap / 1024 + 2)) * sizeof(int)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->scratch, 128 * sizeof(int)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->buf, 6 * cap * sizeof(double)), "ws");
	pinc_check(pinc_hip_malloc((void **)&ws->bufNe, cap + 16), "ws");
}

static void ws_free(pinc_extract_ws_t *ws) {
	pinc_hip_free(ws->tail);
	pinc_hip_free(ws->holes);
	pinc_hip_free(ws->order);
	pinc_hip_free(ws->blockHist);
	pinc_hip_free(ws->scratch);
	pinc_hip_free(ws->buf);
	pinc_hip_free(ws->bufNe);
	memset(ws, 0, sizeof(*ws));
}

/* grow the emigrant buffers of species s to hold at least n emigrants */
void pinc_pop_grow_ws(Population *pop, int s, long n) {
	PincDevPop *dv = pop->dev;
	int *chunkOffset = dv->ws[s].chunkOffset, *scanWork = dv->ws[s].scanWork;
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), "grow sync");
	ws_free(&dv->ws[s]);
	ws_alloc(&dv->ws[s], n + n / 4 + 1024);
	dv->ws[s].chunkOffset = chunkOffset;
	dv->ws[s].scanWork = scanWork;
}

Population *pAlloc(const dictionary *ini) {
	pinc_ctx_require();
	int ns = iniGetInt(ini, "population:nSpecies");
	int nd = iniGetInt(ini, "grid:nDims");
	long *tot = iniGetLongIntArr(ini, "population:nAlloc", ns);
	Population *p = calloc(1, sizeof(*p));
	p->nSpecies = ns;
	p->nDims = nd;
	p->iStart = calloc(ns + 1, sizeof(long));
	p->iStop = calloc(ns, sizeof(long));
	for (int s = 1; s <= ns; s++) {
		long nAlloc = (long)ceil((double)tot[s - 1] / g_pinc.nranks);
		if (nAlloc * g_pinc.nranks != tot[s - 1])
			msg(WARNING, "increased number of allocated particles to get integer per computing node");
		p->iStart[s] = p->iStart[s - 1] + nAlloc;
	}
	for (int s = 0; s < ns; s++) p->iStop[s] = p->iStart[s];
	free(tot);
	p->charge = iniGetDoubleArr(ini, "population:charge", ns);
	p->mass = iniGetDoubleArr(ini, "population:mass", ns);
	p->kinEnergy = calloc(ns + 1, sizeof(double));
	p->potEnergy = calloc(ns + 1, sizeof(double));

	PincDevPop *dv = calloc(1, sizeof(*dv));
	long cap = p->iStart[ns];
	dv->cap = cap;
	dv->p.nd = nd;
	dv->p.nSpecies = ns;
	for (int d = 0; d < nd; d++) {
		pinc_check(pinc_hip_malloc((void **)&dv->p.x[d], cap * sizeof(double)), "pAlloc pos");
		pinc_check(pinc_hip_malloc((void **)&dv->p.v[d], cap * sizeof(double)), "pAlloc vel");
	}
	pinc_check(pinc_hip_malloc((void **)&dv->flags, cap + 16), "pAlloc flags");
	if (iniHas(ini, "population:layout")) {
		char *lay = iniGetStr(ini, "population:layout");
		if (!strcmp(lay, "tiled")) dv->tiled = 1;
		else if (strcmp(lay, "reference")) msg(ERROR, "population:layout must be reference or tiled, not %s", lay);
		free(lay);
	}
	dv->fused = iniHas(ini, "population:fused") ? iniGetInt(ini, "population:fused") : 1;
	if (dv->tiled) {
		dv->sortInterval = iniHas(ini, "population:sortInterval") ? iniGetInt(ini, "population:sortInterval") : 8;
		if (dv->sortInterval < 1) msg(ERROR, "population:sortInterval must be >= 1");
		dv->tileWidth = nd == 3 ? 4 : (nd == 2 ? 8 : 32);
		/* population:tileWidth (or PINC_TILE_WIDTH, experiments): cells per
		 * tile edge, a power of two */
		if (iniHas(ini, "population:tileWidth")) dv->tileWidth = iniGetInt(ini, "population:tileWidth");
		if (getenv("PINC_TILE_WIDTH") && *getenv("PINC_TILE_WIDTH")) dv->tileWidth = atoi(getenv("PINC_TILE_WIDTH"));
		if (dv->tileWidth < 2 || (dv->tileWidth & (dv->tileWidth - 1)))
			msg(ERROR, "population:tileWidth must be a power of two >= 2, not %d", dv->tileWidth);
		for (int s = 0; s < PINC_MAX_SPECIES; s++) dv->cellValid[s] = -1;
	}
	/* tiled + fused: the counting sort rides in every sortInterval-th push
	 * (population:sortInPush=1, default) or runs as a pass of its own (0) */
	dv->sorted = dv->tiled && dv->fused &&
	             (iniHas(ini, "population:sortInPush") ? iniGetInt(ini, "population:sortInPush") : 1);
	if (dv->sorted) {
		dv->sortFraction = iniHas(ini, "population:sortFraction") ? iniGetDouble(ini, "population:sortFraction") : 0.0;
		dv->sortMax = iniHas(ini, "population:sortMax") ? iniGetInt(ini, "population:sortMax") : 32;
		if (dv->sortFraction < 0 || dv->sortMax < 1) msg(ERROR, "population:sortFraction/sortMax out of range");
		dv->sortSpread = iniHas(ini, "population:sortSpread") ? iniGetDouble(ini, "population:sortSpread") : 0.0;
		if (dv->sortSpread < 0) msg(ERROR, "population:sortSpread out of range");
		if (dv->sortFraction > 0) {
			/* moved and spread counters and the kinetic-energy sums in one
			 * block: one read per push */
			pinc_check(pinc_hip_malloc((void **)&dv->movedCnt, 4 * PINC_MAX_SPECIES * sizeof(unsigned long long)),
			           "pAlloc moved");
			dv->spreadCnt = dv->movedCnt + PINC_MAX_SPECIES;
			dv->emigCnt = dv->movedCnt + 3 * PINC_MAX_SPECIES;
			for (int s = 0; s < PINC_MAX_SPECIES; s++) dv->sortNext[s] = 1;
		}
	}
	if (dv->tiled || dv->fused) {
		for (int d = 0; d < nd; d++) {
			pinc_check(pinc_hip_malloc((void **)&dv->altX[d], cap * sizeof(double)), "pAlloc pos (tiled)");
			pinc_check(pinc_hip_malloc((void **)&dv->altV[d], cap * sizeof(double)), "pAlloc vel (tiled)");
		}
	}
	long maxS = 0;
	dv->chunkBase[0] = 0;
	for (int s = 0; s < ns; s++) {
		long capS = p->iStart[s + 1] - p->iStart[s];
		if (capS > maxS) maxS = capS;
		dv->chunkBase[s + 1] = dv->chunkBase[s] + capS / PINC_CHUNK + 2;
	}
	long nChunks = maxS / PINC_CHUNK + 2;
	int *chunkOffset = NULL;
	pinc_check(pinc_hip_malloc((void **)&dv->chunkCount, dv->chunkBase[ns] * sizeof(int)), "pAlloc chunks");
	/* one KE partial per push block (PINC_CHUNK/2 particles by default, at
	 * least PINC_CHUNK/8) */
	pinc_check(pinc_hip_malloc((void **)&dv->kePartial, (maxS / (PINC_CHUNK / 8) + 16) * sizeof(double)), "pAlloc ke");
	long scanWork = 2 * (nChunks / 4096 + 1) + 1;
	pinc_check(pinc_hip_malloc((void **)&chunkOffset, (nChunks + 1 + scanWork) * sizeof(int)), "pAlloc chunks");
	for (int s = 0; s < ns; s++) {
		long capS = p->iStart[s + 1] - p->iStart[s];
		long ecap = capS / 64;
		if (ecap < 65536) ecap = 65536;
		ws_alloc(&dv->ws[s], ecap);
		dv->ws[s].chunkOffset = chunkOffset;
		dv->ws[s].scanWork = chunkOffset + nChunks + 1;
	}
	double qm[PINC_MAX_SPECIES] = {0}, mq[PINC_MAX_SPECIES] = {0};
	for (int s = 0; s < ns; s++) {
		qm[s] = p->charge[s] / p->mass[s];
		mq[s] = p->mass[s] / p->charge[s];
	}
	pinc_check(pinc_hip_malloc((void **)&dv->qm, sizeof(qm)), "pAlloc qm");
	pinc_check(pinc_hip_malloc((void **)&dv->mq, sizeof(mq)), "pAlloc mq");
	pinc_check(pinc_hip_h2d(dv->qm, qm, sizeof(qm), g_pinc.stream), "pAlloc qm");
	pinc_check(pinc_hip_h2d(dv->mq, mq, sizeof(mq), g_pinc.stream), "pAlloc mq");
	dv->geom = pinc_geom_current();
	p->dev = dv;
	/* the bound the kernels check velocities against (pVelAssertMax) */
	g_pinc.maxVel = iniHas(ini, "population:maxVel") ? iniGetDouble(ini, "population:maxVel") : INFINITY;
	return p;
}

void pinc_pop_flush_host(const Population *pop) {
	if (pop->dev->hostDirty) pSyncToDevice((Population *)pop);
}

/* population.c:342-365 and 316-340.  On the device the two checks run where
 * the kernels touch the particles: the velocity bound in the kick of the
 * fused push (or the move), the local frame after the move's periodic shift;
 * both set bits of one assert word.  The calls main.c makes each step read
 * that word (4 bytes) and end the run with msg(ERROR) as the reference does.
 * A velocity the move has not yet seen is reported by the
 * pPosAssertInLocalFrame of the same step, before anything deposits it.  A
 * bound other than the kernels' (population:maxVel) is adopted from this call
 * on, and the velocities present now are checked against it here. */
static int assert_word(void) {
	int err = 0;
	g_pinc.errRead = g_pinc.errSerial;
	pinc_check(pinc_hip_d2h(&err, g_pinc.dErr, sizeof(int), g_pinc.stream), "assert word");
	return err;
}

void pVelAssertMax(const Population *pop, double max) {
	PincDevPop *dv = pop->dev;
	const int fresh = dv->hostDirty; /* velocities no kernel has checked yet */
	pinc_pop_flush_host(pop);
	if (max != g_pinc.maxVel || fresh) {
		g_pinc.maxVel = max;
		pinc_pop_t p = pinc_devpop(pop);
		/* a pending sorted push keeps the kicked velocities in altV (same
		 * ranges, slot order) */
		if (dv->pending && dv->pendingSorted)
			for (int d = 0; d < pop->nDims; d++) p.v[d] = dv->altV[d];
		for (int s = 0; s < pop->nSpecies; s++)
			pinc_check(pinc_hip_vel_assert(p, s, max, g_pinc.dErr, g_pinc.stream), "pVelAssertMax");
		g_pinc.errSerial++;
	}
	if (assert_word() & 1)
		msg(ERROR, "Particle travels too fast (population:maxVel=%g exceeded, population.c:342-365)", max);
}

void pPosAssertInLocalFrame(const Population *pop, const Grid *grid) {
	(void)grid; /* the bounds are MpiInfo's thresholds, from the same grid size */
	int err = assert_word();
	if (err & 2) msg(ERROR, "Particle is out of bounds after migration (population.c:316-340)");
	if (err & 1) msg(ERROR, "Particle travels too fast (population:maxVel exceeded, population.c:342-365)");
	(void)pop;
}

void pFree(Population *p) {
	if (!p) return;
	PincDevPop *dv = p->dev;
	pinc_pending_unregister(p);
	if (dv) {
		pinc_pop_settle(p); /* (the copy into hostCnt has landed) */
		pinc_hip_host_free(dv->hostCnt);
		if (dv->cntEvent) pinc_hip_event_destroy(dv->cntEvent);
		/* main.c:297-298 frees the population before the objects */
		if (dv->objOwner) pinc_obj_forget_pop(dv->objOwner);
		for (int d = 0; d < p->nDims; d++) {
			pinc_hip_free(dv->p.x[d]);
			pinc_hip_free(dv->p.v[d]);
		}
		pinc_hip_free(dv->flags);
		for (int d = 0; d < 3; d++) {
			pinc_hip_free(dv->altX[d]);
			pinc_hip_free(dv->altV[d]);
		}
		for (int s = 0; s < PINC_MAX_SPECIES; s++) {
			pinc_hip_free(dv->rhoS[s]);
			pinc_hip_free(dv->keyCnt[s]);
			pinc_hip_free(dv->keyNext[s]);
			pinc_hip_free(dv->keyCur[s]);
			pinc_hip_free(dv->keyWork[s]);
		}
		pinc_hip_free(dv->movedCnt);
		for (int s = 0; s < PINC_MAX_SPECIES; s++) pinc_hip_free(dv->sortWork[s]);
		pinc_hip_free(dv->chunkCount);
		pinc_hip_free(dv->ws[0].chunkOffset);
		for (int s = 0; s < p->nSpecies; s++) ws_free(&dv->ws[s]);
		pinc_hip_free(dv->qm);
		pinc_hip_free(dv->mq);
		pinc_hip_free(dv->kePartial);
		for (int k = 0; k < 2; k++) {
			pinc_hip_free(dv->sendBuf[k]);
			pinc_hip_free(dv->recvBuf[k]);
		}
		free(dv);
	}
	free(p->pos);
	free(p->vel);
	free(p->iStart);
	free(p->iStop);
	free(p->charge);
	free(p->mass);
	free(p->kinEnergy);
	free(p->potEnergy);
	free(p);
	free(g_hostIds);
	g_hostIds = NULL;
}

pinc_pop_t pinc_devpop(const Population *pop) {
	pinc_pop_t p = pop->dev->p;
	for (int s = 0; s <= pop->nSpecies; s++) p.iStart[s] = pop->iStart[s];
	for (int s = 0; s < pop->nSpecies; s++) p.iStop[s] = pop->iStop[s];
	return p;
}

static void host_arrays(Population *p) {
	long n = (long)p->nDims * p->iStart[p->nSpecies];
	if (!p->pos) p->pos = calloc(n ? n : 1, sizeof(double));
	if (!p->vel) p->vel = calloc(n ? n : 1, sizeof(double));
	if (!g_hostIds) g_hostIds = calloc(p->iStart[p->nSpecies] + 1, sizeof(long));
}

void pToLocalFrame(Population *p, const MpiInfo *m) {
	host_arrays(p);
	int nd = p->nDims;
	for (int s = 0; s < p->nSpecies; s++)
		for (long i = p->iStart[s]; i < p->iStop[s]; i++)
			for (int d = 0; d < nd; d++) p->pos[i * nd + d] -= m->offset[d];
}

void pToGlobalFrame(Population *p, const MpiInfo *m) {
	host_arrays(p);
	int nd = p->nDims;
	for (int s = 0; s < p->nSpecies; s++)
		for (long i = p->iStart[s]; i < p->iStop[s]; i++)
			for (int d = 0; d < nd; d++) p->pos[i * nd + d] += m->offset[d];
}

static void globalSize(const dictionary *ini, int nd, int *L, long *V) {
	int *ts = iniGetIntArr(ini, "grid:trueSize", nd);
	int *ns = iniGetIntArr(ini, "grid:nSubdomains", nd);
	long v = 1;
	for (int d = 0; d < nd; d++) {
		L[d] = ns[d] * ts[d];
		v *= L[d];
	}
	*V = v;
	free(ts);
	free(ns);
}

void pPosLattice(const dictionary *ini, Population *p, const MpiInfo *m) {
	host_arrays(p);
	int nd = p->nDims;
	long *nPart = iniGetLongIntArr(ini, "population:nParticles", p->nSpecies);
	int L[3];
	long V;
	globalSize(ini, nd, L, &V);
	for (int s = 0; s < p->nSpecies; s++) {
		double l = pow(V / (double)nPart[s], 1.0 / nd);
		long k = p->iStart[s];
		for (long i = 0; i < nPart[s]; i++) {
			double x[3], lin = l * i;
			for (int d = 0; d < nd; d++) {
				x[d] = fmod(lin, L[d]);
				lin /= L[d];
			}
			int ok = 0;
			for (int d = 0; d < nd; d++) ok += (m->subdomain[d] == (int)(m->posToSubdomain[d] * x[d]));
			if (ok == nd) {
				if (k >= p->iStart[s + 1])
					msg(ERROR, "allocated only %li particles of specie %i per node", p->iStart[s + 1] - p->iStart[s], s);
				for (int d = 0; d < nd; d++) p->pos[k * nd + d] = x[d];
				g_hostIds[k] = i;
				k++;
			}
		}
		p->iStop[s] = k;
	}
	pToLocalFrame(p, m);
	free(nPart);
	p->dev->hostDirty = 1;
}

void pPosPerturb(const dictionary *ini, Population *p, const MpiInfo *m) {
	int nd = p->nDims, ns = p->nSpecies;
	double *amp = iniGetDoubleArr(ini, "population:perturbAmplitude", nd * ns);
	double *mode = iniGetDoubleArr(ini, "population:perturbMode", nd * ns);
	int L[3];
	long V;
	globalSize(ini, nd, L, &V);
	pToGlobalFrame(p, m);
	for (int s = 0; s < ns; s++)
		for (long i = p->iStart[s]; i < p->iStop[s]; i++)
			for (int d = 0; d < nd; d++) {
				double theta = 2.0 * M_PI * mode[s * nd + d] * p->pos[i * nd + d] / L[d];
				p->pos[i * nd + d] += amp[s * nd + d] * cos(theta);
			}
	pToLocalFrame(p, m);
	free(amp);
	free(mode);
	p->dev->hostDirty = 1;
}

void pVelZero(Population *p) {
	host_arrays(p);
	int nd = p->nDims;
	for (int s = 0; s < p->nSpecies; s++)
		for (long i = p->iStart[s]; i < p->iStop[s]; i++)
			for (int d = 0; d < nd; d++) p->vel[i * nd + d] = 0;
	p->dev->hostDirty = 1;
}

static unsigned long long mix64(unsigned long long z) {
	z += 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}
static double uni(unsigned long long seed, unsigned long long c) {
	unsigned long long x = mix64(seed ^ mix64(c));
	return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}
static double gauss(unsigned long long seed, unsigned long long c) {
	double u1 = uni(seed, 2 * c), u2 = uni(seed, 2 * c + 1);
	return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

void pVelMaxwell(const dictionary *ini, Population *p, unsigned long long seed) {
	host_arrays(p);
	int nd = p->nDims, ns = p->nSpecies;
	double *drift = iniGetDoubleArr(ini, "population:drift", ns);
	double *vth = iniGetDoubleArr(ini, "population:thermalVelocity", ns);
	for (int s = 0; s < ns; s++)
		for (long i = p->iStart[s]; i < p->iStop[s]; i++) {
			unsigned long long c = (((unsigned long long)s << 40) | (unsigned long long)g_hostIds[i]) * 3ULL;
			for (int d = 0; d < nd; d++) p->vel[i * nd + d] = drift[s] + vth[s] * gauss(seed, c + d);
		}
	free(drift);
	free(vth);
	p->dev->hostDirty = 1;
}

void pSumKinEnergy(Population *p) {
	pinc_pop_settle(p); /* a fused puAcc3D1KE's sums */
	int ns = p->nSpecies;
	p->kinEnergy[ns] = 0;
	for (int s = 0; s < ns; s++) p->kinEnergy[ns] += p->kinEnergy[s];
}

void pSyncToHost(Population *p) {
	if (p->dev->hostDirty && p->pos) return; /* the host mirror is the truth */
	host_arrays(p);
	int nd = p->nDims;
	PincDevPop *dv = p->dev;
	for (int s = 0; s < p->nSpecies; s++) {
		long a = p->iStart[s], n = p->iStop[s] - a;
		if (n <= 0) continue;
		double *tmp = malloc(n * sizeof(double));
		double *dtmp = NULL;
		/* a sorted fused push is pending: the kicked velocities in the current
		 * order come from pinc_pending_vel */
		if (dv->pending && dv->pendingSorted) {
			pinc_check(pinc_hip_malloc((void **)&dtmp, nd * n * sizeof(double)), "pSyncToHost tmp");
			double *dst[3] = {dtmp, dtmp + n, dtmp + 2 * n};
			pinc_pending_vel(p, s, dst);
		}
		for (int d = 0; d < nd; d++) {
			pinc_check(pinc_hip_d2h(tmp, dv->p.x[d] + a, n * sizeof(double), g_pinc.stream), "pSyncToHost");
			for (long i = 0; i < n; i++) p->pos[(a + i) * nd + d] = tmp[i];
			const double *vsrc = dtmp ? dtmp + d * n : dv->p.v[d] + a;
			pinc_check(pinc_hip_d2h(tmp, vsrc, n * sizeof(double), g_pinc.stream), "pSyncToHost");
			for (long i = 0; i < n; i++) p->vel[(a + i) * nd + d] = tmp[i];
		}
		pinc_hip_free(dtmp);
		free(tmp);
	}
}

void pSyncToDevice(Population *p) {
	if (!p->pos) msg(ERROR, "pSyncToDevice without host particles");
	int nd = p->nDims;
	PincDevPop *dv = p->dev;
	pinc_pop_settle(p); /* before the schedule is reset below */
	dv->hostDirty = 0;
	/* new particles: a pending fused move and its deposits no longer apply */
	dv->pending = dv->pendingSorted = dv->depValid = dv->depExtracted = 0;
	dv->everSorted = 0;
	for (int s = 0; s < PINC_MAX_SPECIES; s++) {
		dv->cntValid[s] = 0;
		dv->sortNext[s] = 1;
		dv->movedFrac[s] = dv->lastRate[s] = 0.0;
		dv->sinceSort[s] = 0;
	}
	/* new particle order: the cell ranges of the last tile sort no longer apply */
	for (int s = 0; s < PINC_MAX_SPECIES; s++) dv->cellValid[s] = -1;
	for (int s = 0; s < p->nSpecies; s++) {
		long a = p->iStart[s], n = p->iStop[s] - a;
		if (n <= 0) continue;
		double *tmp = malloc(n * sizeof(double));
		for (int d = 0; d < nd; d++) {
			for (long i = 0; i < n; i++) tmp[i] = p->pos[(a + i) * nd + d];
			pinc_check(pinc_hip_h2d(dv->p.x[d] + a, tmp, n * sizeof(double), g_pinc.stream), "pSyncToDevice");
			for (long i = 0; i < n; i++) tmp[i] = p->vel[(a + i) * nd + d];
			pinc_check(pinc_hip_h2d(dv->p.v[d] + a, tmp, n * sizeof(double), g_pinc.stream), "pSyncToDevice");
		}
		free(tmp);
	}
	dv->flagsValid = 0;
}

void pInitDevice(const dictionary *ini, Population *p, const MpiInfo *m, int perturb, int maxwell,
                 unsigned long long seed) {
	int nd = p->nDims, ns = p->nSpecies;
	long *nPart = iniGetLongIntArr(ini, "population:nParticles", ns);
	double *amp = iniGetDoubleArr(ini, "population:perturbAmplitude", nd * ns);
	double *mode = iniGetDoubleArr(ini, "population:perturbMode", nd * ns);
	double *drift = iniGetDoubleArr(ini, "population:drift", ns);
	double *vth = iniHas(ini, "population:thermalVelocity")
	                  ? iniGetDoubleArr(ini, "population:thermalVelocity", ns)
	                  : calloc(ns, sizeof(double));
	int L[3];
	long V;
	globalSize(ini, nd, L, &V);
	pinc_geom_t g = p->dev->geom;
	for (int s = 0; s < ns; s++) {
		double l = pow(V / (double)nPart[s], 1.0 / nd);
		pinc_pop_t dp = pinc_devpop(p);
		long n = 0;
		pinc_check(pinc_hip_init_species(dp, s, g, nPart[s], l, m->subdomain, m->nSubdomains, m->offset,
		                                 amp + s * nd, mode + s * nd, perturb, maxwell, drift[s], vth[s],
		                                 seed, &n, g_pinc.stream),
		           "pInitDevice");
		p->iStop[s] = p->iStart[s] + n;
	}
	p->dev->flagsValid = 0;
	p->dev->hostDirty = 0;
	free(nPart);
	free(amp);
	free(mode);
	free(drift);
	free(vth);
}
