/*
 * pinc_pusher.c -- particle operators of the MI355X PINC hot path (host C).
 * Same names, signatures and _set selectors as src/pusher.c; each launches
 * the gfx950 kernels of libpinc_hip on the device twin.
 *
 *   puMove                 pusher.c:86-119 (+ fused neighbour classification)
 *   puAcc3D1(KE)/ND1(KE)   pusher.c:147-308
 *   puDistr3D1/ND1         pusher.c:512-638
 *   puExtractEmigrants*    pusher.c:782-910
 *   puMigrate              pusher.c:914-1035: one rank imports its own
 *                          emigrants (all neighbours are itself); with a slab
 *                          decomposition the z+-1 payloads travel over RCCL
 *   puNeighborToRank etc.  pusher.c:1181-1232
 *   _set sanity checks     pusher.c:1047-1087
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <math.h>

void pinc_pop_grow_ws(Population *pop, int s, long n);

/* ------------------------------------------------------------- sanity -- */
static void puSanity(dictionary *ini, const char *name, int dim, int order) {
	int nd = iniGetInt(ini, "grid:nDims");
	int *ng = iniGetIntArr(ini, "grid:nGhostLayers", 2 * nd);
	double *th = iniGetDoubleArr(ini, "grid:thresholds", 2 * nd);
	int minL = ng[0];
	double mn = th[0], mx = th[0];
	for (int i = 1; i < 2 * nd; i++) {
		if (ng[i] < minL) minL = ng[i];
		if (th[i] < mn) mn = th[i];
		if (th[i] > mx) mx = th[i];
	}
	if (nd != dim && dim != 0) msg(ERROR, "%s only supports grid:nDims=%d", name, dim);
	if (minL < 1) msg(ERROR, "%s requires grid:nGhostLayers >=%d", name, order ? 1 : 0);
	double reqMin = order == 0 ? -0.5 : (order == 1 ? 0 : 0.5);
	if (mn < reqMin) msg(ERROR, "%s requires grid:thresholds >=%.1f", name, reqMin);
	if (mx > minL - 0.5) msg(ERROR, "%s requires grid:thresholds <= grid:nGhostLayers - 0.5", name);
	free(ng);
	free(th);
}

funPtr puAcc3D1_set(dictionary *ini) { puSanity(ini, "puAcc3D1", 3, 1); return (funPtr)puAcc3D1; }
funPtr puAcc3D1KE_set(dictionary *ini) { puSanity(ini, "puAcc3D1KE", 3, 1); return (funPtr)puAcc3D1KE; }
funPtr puAccND1_set(dictionary *ini) { puSanity(ini, "puAccND1", 0, 1); return (funPtr)puAccND1; }
funPtr puAccND1KE_set(dictionary *ini) { puSanity(ini, "puAccND1KE", 0, 1); return (funPtr)puAccND1KE; }
/* Boris (puBoris3D1/KE, pusher.c:394-505), an extension: the reference's
 * version rotates the wrong particle (fact 7) and main.c does not offer it.
 * Selected as methods:acc=puBoris3D1KE; the rotation parameters come from
 * the normalised ini at the first push (select runs before uNormalize,
 * main.c:55-85), and the initial half step halves E and T (S recomputed for
 * the halved T, so the half rotation stays norm-preserving). */
static struct {
	const dictionary *ini;
	int ready, half;
	double T[3 * PINC_MAX_SPECIES], S[3 * PINC_MAX_SPECIES];
	double Th[3 * PINC_MAX_SPECIES], Sh[3 * PINC_MAX_SPECIES];
} g_boris;

void puGet3DRotationParameters(dictionary *ini, double *T, double *S) {
	int nDims = iniGetInt(ini, "grid:nDims");
	int nSpecies = iniGetInt(ini, "population:nSpecies");
	if (nDims != 3) msg(ERROR, "Boris rotation parameters need grid:nDims=3");
	double *BExt = iniGetDoubleArr(ini, "fields:BExt", nDims);
	double *charge = iniGetDoubleArr(ini, "population:charge", nSpecies);
	double *mass = iniGetDoubleArr(ini, "population:mass", nSpecies);
	for (int s = 0; s < nSpecies; s++) {
		double factor = 0.5 * charge[s] / mass[s];
		double denom = 1;
		for (int p = 0; p < 3; p++) {
			T[3 * s + p] = factor * BExt[p];
			denom += T[3 * s + p] * T[3 * s + p];
		}
		double mul = 2.0 / denom;
		for (int p = 0; p < 3; p++) S[3 * s + p] = mul * T[3 * s + p];
	}
	free(BExt);
	free(charge);
	free(mass);
}

static void boris(Population *pop, Grid *E, const double *T, const double *S, int ke);
static void boris_params(void) {
	if (g_boris.ready) return;
	if (!g_boris.ini) msg(ERROR, "Boris pusher used without puBoris3D1*_set");
	puGet3DRotationParameters((dictionary *)g_boris.ini, g_boris.T, g_boris.S);
	for (int i = 0; i < 3 * PINC_MAX_SPECIES; i += 3) {
		double denom = 1;
		for (int p = 0; p < 3; p++) {
			g_boris.Th[i + p] = 0.5 * g_boris.T[i + p];
			denom += g_boris.Th[i + p] * g_boris.Th[i + p];
		}
		for (int p = 0; p < 3; p++) g_boris.Sh[i + p] = 2.0 / denom * g_boris.Th[i + p];
	}
	g_boris.ready = 1;
}
static void boris_selected(Population *pop, Grid *E, int ke) {
	boris_params();
	if (g_boris.half) boris(pop, E, g_boris.Th, g_boris.Sh, ke);
	else boris(pop, E, g_boris.T, g_boris.S, ke);
}
static void boris_sel(Population *pop, Grid *E) { boris_selected(pop, E, 0); }
static void boris_sel_ke(Population *pop, Grid *E) { boris_selected(pop, E, 1); }
void pinc_boris_half_step(int on) { g_boris.half = on; }
int pinc_boris_selected(funPtr acc) { return acc == (funPtr)boris_sel || acc == (funPtr)boris_sel_ke; }
funPtr puBoris3D1_set(dictionary *ini) {
	puSanity(ini, "puBoris3D1", 3, 1);
	g_boris.ini = ini;
	g_boris.ready = 0;
	return (funPtr)boris_sel;
}
funPtr puBoris3D1KE_set(dictionary *ini) {
	puSanity(ini, "puBoris3D1KE", 3, 1);
	g_boris.ini = ini;
	g_boris.ready = 0;
	return (funPtr)boris_sel_ke;
}
/* order 0 (nearest grid point, pusher.c:310-391, 640-668); puAccND0_set
 * returns the KE variant, as the reference does (pusher.c:356-358) */
funPtr puAccND0_set(dictionary *ini) { puSanity(ini, "puAccND0", 0, 0); return (funPtr)puAccND0KE; }
funPtr puAccND0KE_set(dictionary *ini) { puSanity(ini, "puAccND0KE", 0, 0); return (funPtr)puAccND0KE; }
funPtr puDistrND0_set(dictionary *ini) { puSanity(ini, "puDistrND0", 0, 0); return (funPtr)puDistrND0; }
funPtr puDistr3D1_set(dictionary *ini) { puSanity(ini, "puDistr3D1", 3, 1); return (funPtr)puDistr3D1; }
funPtr puDistrND1_set(dictionary *ini) { puSanity(ini, "puDistrND1", 0, 1); return (funPtr)puDistrND1; }
funPtr puExtractEmigrants3D_set(dictionary *ini) {
	if (iniGetInt(ini, "grid:nDims") != 3) msg(ERROR, "puExtractEmigrants3D requires grid:nDims=3");
	return (funPtr)puExtractEmigrants3D;
}
funPtr puExtractEmigrantsND_set(dictionary *ini) {
	(void)ini;
	return (funPtr)puExtractEmigrantsND;
}

/* ----------------------------------------------------------- neighbours -- */
int puNeighborToReciprocal(int neighbor, int nDims) {
	int r = 0;
	for (int d = 0; d < nDims; d++) {
		r += (2 - (neighbor % 3)) * pinc_ipow3(d);
		neighbor /= 3;
	}
	return r;
}

int puNeighborToRank(MpiInfo *m, int neighbor) {
	int rank = 0;
	for (int d = 0; d < m->nDims; d++) {
		int n = (neighbor % 3) - 1;
		neighbor /= 3;
		n = (m->subdomain[d] + n + m->nSubdomains[d]) % m->nSubdomains[d];
		rank += n * m->nSubdomainsProd[d];
	}
	return rank;
}

int puRankToNeighbor(MpiInfo *m, int rank) {
	int neighbor = 0;
	for (int d = 0; d < m->nDims; d++) {
		int n = rank % m->nSubdomains[d];
		n = (n - m->subdomain[d] + 1 + m->nSubdomains[d]) % m->nSubdomains[d];
		rank /= m->nSubdomains[d];
		neighbor += n * pinc_ipow3(d);
	}
	return neighbor;
}

/* ---------------------------------------------------------------- move -- */
/* tiled layout: counting sort by tile into the alternate arrays, then swap */
static void sort_tiles(Population *pop) {
	PincDevPop *dv = pop->dev;
	pinc_pop_t p = pinc_devpop(pop), out = p;
	for (int d = 0; d < pop->nDims; d++) {
		out.x[d] = dv->altX[d];
		out.v[d] = dv->altV[d];
	}
	for (int s = 0; s < pop->nSpecies; s++) {
		long nKeys = 0;
		int rc = pinc_hip_sort_tiles(p, out, s, dv->geom, dv->tileWidth, dv->sortWork[s], dv->sortWorkCap[s], &nKeys,
		                             g_pinc.stream);
		long need = 2 * (nKeys + 1) + 2 * (nKeys / 4096 + 1) + 1;
		if (rc && need > dv->sortWorkCap[s]) {
			pinc_hip_free(dv->sortWork[s]);
			dv->sortWorkCap[s] = need;
			pinc_check(pinc_hip_malloc((void **)&dv->sortWork[s], need * sizeof(int)), "sort work");
			rc = pinc_hip_sort_tiles(p, out, s, dv->geom, dv->tileWidth, dv->sortWork[s], dv->sortWorkCap[s], &nKeys,
			                         g_pinc.stream);
		}
		pinc_check(rc, "sort tiles");
		dv->sortKeys = nKeys;
		dv->cellValid[s] = pop->iStop[s] - pop->iStart[s];
	}
	for (int d = 0; d < pop->nDims; d++) {
		double *t = dv->p.x[d];
		dv->p.x[d] = dv->altX[d];
		dv->altX[d] = t;
		t = dv->p.v[d];
		dv->p.v[d] = dv->altV[d];
		dv->altV[d] = t;
	}
}

/* tiled layout: re-sort every sortInterval moves (before moving) */
static void maybe_sort(Population *pop) {
	PincDevPop *dv = pop->dev;
	if (dv->tiled && dv->moves++ % dv->sortInterval == 0) sort_tiles(pop);
}

/* tiled layout: rank-local periodic crossings are wrapped in place */
static int wrap_mask(const Population *pop) {
	int nd = pop->nDims;
	return !pop->dev->tiled ? 0 : (g_pinc.nranks == 1 ? (1 << nd) - 1 : (1 << (nd - 1)) - 1);
}

/* ------------------------------------------------------------- flags -- */
/* One flag byte per particle slot: its neighbour code after the last
 * classification, which the extraction reads (pinc_hip_extract).  Only the
 * leavers' codes differ from the centre, and the extraction puts theirs back
 * to the centre.  So when all of species s's range holds the centre
 * (PINC_FLAGS_CLEAN), a push writes only its leavers' flags: at one rank,
 * where every dimension wraps in place, no flag at all instead of 1 B per
 * particle.  A write that leaves flags behind the extraction cannot reach
 * (a second push before an extraction, a range that shrank in between) makes
 * the state unknown, and the next push first sets the range to the centre. */
static int flag_center(const Population *pop) {
	int c = 0;
	for (int d = 0, p = 1; d < pop->nDims; d++, p *= 3) c += p;
	return c;
}

/* before a launch that writes species s's flags: 1 if it may write only the
 * leavers' (sparseOk: a push), 0 if it writes every live particle's */
int pinc_flags_before_write(Population *pop, int s, int sparseOk) {
	PincDevPop *dv = pop->dev;
	const long n = pop->iStop[s] - pop->iStart[s];
	if (sparseOk && g_pinc.flagsSparse) {
		if (dv->flagState[s] != PINC_FLAGS_CLEAN) {
			const long a = pop->iStart[s], len = pop->iStart[s + 1] - a;
			if (len > 0)
				pinc_check(pinc_hip_memset(dv->flags + a, flag_center(pop), (unsigned long)len, g_pinc.stream),
				           "flags to the centre");
		}
		dv->flagState[s] = PINC_FLAGS_PENDING;
		dv->flagN[s] = n;
		return 1;
	}
	/* a full write covers [0, n): the flags of an earlier write survive only
	 * beyond n */
	if (dv->flagState[s] == PINC_FLAGS_CLEAN || (dv->flagState[s] == PINC_FLAGS_PENDING && n >= dv->flagN[s])) {
		dv->flagState[s] = PINC_FLAGS_PENDING;
		dv->flagN[s] = n;
	} else {
		dv->flagState[s] = PINC_FLAGS_UNKNOWN;
	}
	return 0;
}

/* after pinc_hip_extract of species s over its nBefore live particles: every
 * flagged particle was extracted and its flag put back */
void pinc_flags_after_extract(Population *pop, int s, long nBefore) {
	PincDevPop *dv = pop->dev;
	if (dv->flagState[s] == PINC_FLAGS_PENDING)
		dv->flagState[s] = nBefore >= dv->flagN[s] ? PINC_FLAGS_CLEAN : PINC_FLAGS_UNKNOWN;
}

/* tiled + fused: key counts of the current positions and scratch */
static void ensure_keys(Population *pop) {
	PincDevPop *dv = pop->dev;
	long nk = pinc_hip_tile_keys(dv->geom, dv->tileWidth);
	if (dv->nKeys == nk && dv->keyCnt[0]) return;
	for (int s = 0; s < PINC_MAX_SPECIES; s++) {
		pinc_hip_free(dv->keyCnt[s]);
		pinc_hip_free(dv->keyNext[s]);
		pinc_hip_free(dv->keyCur[s]);
		pinc_hip_free(dv->keyWork[s]);
		dv->keyCnt[s] = dv->keyNext[s] = dv->keyCur[s] = dv->keyWork[s] = NULL;
		dv->cntValid[s] = 0;
	}
	for (int s = 0; s < pop->nSpecies; s++) {
		pinc_check(pinc_hip_malloc((void **)&dv->keyCnt[s], (nk + 1) * sizeof(int)), "key counts");
		pinc_check(pinc_hip_malloc((void **)&dv->keyNext[s], (nk + 1) * sizeof(int)), "key counts");
		pinc_check(pinc_hip_malloc((void **)&dv->keyCur[s], (nk + 1) * sizeof(int)), "key cursors");
		pinc_check(pinc_hip_malloc((void **)&dv->keyWork[s], (2 * (nk / 4096 + 1) + 1) * sizeof(int)), "key scan");
	}
	dv->nKeys = nk;
}

static int cmp_double(const void *x, const void *y) {
	const double a = *(const double *)x, b = *(const double *)y;
	return (a > b) - (a < b);
}

/* PINC_TRACE_SORT=2: mean per-block time of each push phase (s_memrealtime,
 * 100 MHz) and the kernel's span */
static void push_phase_report(const unsigned long long *dts, const unsigned long long *ddiag, int nb, int s, int sort,
                              int count, double *const *xout, long i0, long np) {
	unsigned long long *t = malloc((size_t)nb * 8 * sizeof(*t));
	unsigned long long dg[8];
	pinc_check(pinc_hip_d2h(t, dts, (size_t)nb * 8 * sizeof(*t), g_pinc.stream), "push timestamps");
	pinc_check(pinc_hip_d2h(dg, ddiag, sizeof(dg), g_pinc.stream), "push diagnostics");
	double ph[7] = {0};
	unsigned long long t0 = ~0ull, t1 = 0;
	for (int b = 0; b < nb; b++) {
		for (int k = 0; k < 7; k++) ph[k] += (double)(t[b * 8 + k + 1] - t[b * 8 + k]);
		if (t[b * 8] < t0) t0 = t[b * 8];
		if (t[b * 8 + 7] > t1) t1 = t[b * 8 + 7];
	}
	fprintf(stderr, "[pinc] push species %d%s%s: span %.2f ms, per block us: load+box %.2f, lds %.2f, rank %.2f, "
	        "kick/drift %.2f, sorted stores %.2f, count %.2f, deposit %.2f; global slots %.3g, E gathers %.3g "
	        "(wrapped %.3g), charge runs %.3g per block\n", s,
	        sort ? " sort" : "",
	        count ? " count" : "", (t1 - t0) * 1e-5, ph[0] / nb * 1e-2, ph[1] / nb * 1e-2, ph[2] / nb * 1e-2,
	        ph[3] / nb * 1e-2, ph[4] / nb * 1e-2, ph[5] / nb * 1e-2, ph[6] / nb * 1e-2, (double)dg[0] / nb,
	        (double)dg[1] / nb, (double)dg[3] / nb, (double)dg[2] / nb);
	if (sort)
		fprintf(stderr, "[pinc]   sort sub-phases us per block: rank loop %.2f, reservation %.2f\n",
		        dg[4] / (double)nb * 1e-2, ph[2] / nb * 1e-2 - dg[4] / (double)nb * 1e-2);
	/* per XCD (chunk c runs on XCD xcd[c], the push's own placement map):
	 * span from its first block's start to its last block's end, and the
	 * mean number of its blocks between their first and last timestamp */
	if (g_pinc.traceSort > 2) {
		int *xcd = malloc((size_t)nb * sizeof(int));
		pinc_check(pinc_hip_push_xcd_of_chunks(nb, xcd), "push xcd map");
		fprintf(stderr, "[pinc]   xcd span ms / blocks in flight:");
		for (int x = 0; x < 8; x++) {
			unsigned long long a0 = ~0ull, a1 = 0;
			double life = 0;
			for (int b = 0; b < nb; b++) {
				if (xcd[b] != x) continue;
				if (t[b * 8] < a0) a0 = t[b * 8];
				if (t[b * 8 + 7] > a1) a1 = t[b * 8 + 7];
				life += (double)(t[b * 8 + 7] - t[b * 8]);
			}
			fprintf(stderr, " %.2f/%.0f", (a1 - a0) * 1e-5, a1 > a0 ? life / (double)(a1 - a0) : 0.0);
		}
		fprintf(stderr, "\n");
		free(xcd);
		/* block lifetime percentiles (first to last timestamp) */
		double *lv = malloc((size_t)nb * sizeof(*lv));
		for (int b = 0; b < nb; b++) lv[b] = (double)(t[b * 8 + 7] - t[b * 8]) * 1e-2;
		qsort(lv, nb, sizeof(*lv), cmp_double);
		/* the slowest blocks: chunk (position in the species, in chunks),
		 * lifetime, start relative to the launch's first block */
		{
			int top[5] = {-1, -1, -1, -1, -1};
			for (int b = 0; b < nb; b++) {
				const unsigned long long l = t[b * 8 + 7] - t[b * 8];
				for (int k = 0; k < 5; k++) {
					if (top[k] < 0 || l > t[top[k] * 8 + 7] - t[top[k] * 8]) {
						for (int m = 4; m > k; m--) top[m] = top[m - 1];
						top[k] = b;
						break;
					}
				}
			}
			fprintf(stderr, "[pinc]   slowest blocks (chunk of %d: us, start us):", nb);
			for (int k = 0; k < 5 && top[k] >= 0; k++)
				fprintf(stderr, " %d: %.1f, %.1f;", top[k], (t[top[k] * 8 + 7] - t[top[k] * 8]) * 1e-2,
				        (t[top[k] * 8] - t0) * 1e-2);
			fprintf(stderr, "\n");
			/* their particles' cells after the push (unsorted push: same order) */
			const long chunk = pinc_hip_push_chunk();
			double *buf = malloc(chunk * sizeof(double));
			for (int k = 0; k < 5 && top[k] >= 0 && !sort; k++) {
				long b0 = (long)top[k] * chunk, n = b0 + chunk <= np ? chunk : np - b0;
				fprintf(stderr, "[pinc]     chunk %d cells:", top[k]);
				for (int d = 0; d < 3 && xout[d]; d++) {
					pinc_check(pinc_hip_d2h(buf, xout[d] + i0 + b0, n * sizeof(double), g_pinc.stream), "trace read");
					int lo = 1 << 30, hi = -(1 << 30);
					for (long i = 0; i < n; i++) {
						int c = (int)buf[i];
						lo = c < lo ? c : lo;
						hi = c > hi ? c : hi;
					}
					fprintf(stderr, " d%d %d..%d", d, lo, hi);
				}
				fprintf(stderr, "\n");
			}
			free(buf);
		}
		fprintf(stderr, "[pinc]   block us p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n", lv[nb / 10], lv[nb / 2],
		        lv[nb * 9 / 10], lv[nb * 99 / 100], lv[nb - 1]);
		/* phases of the blocks above p90 and below p50 */
		const double p90 = lv[nb * 9 / 10], p50 = lv[nb / 2];
		double hs[7] = {0}, ls[7] = {0};
		int nh = 0, nl = 0;
		for (int b = 0; b < nb; b++) {
			const double l = (double)(t[b * 8 + 7] - t[b * 8]) * 1e-2;
			double *acc = l >= p90 ? hs : (l <= p50 ? ls : NULL);
			if (!acc) continue;
			for (int k = 0; k < 7; k++) acc[k] += (double)(t[b * 8 + k + 1] - t[b * 8 + k]) * 1e-2;
			if (l >= p90) nh++;
			else nl++;
		}
		fprintf(stderr, "[pinc]   phases us, slowest 10%%:");
		for (int k = 0; k < 7; k++) fprintf(stderr, " %.2f", nh ? hs[k] / nh : 0.0);
		fprintf(stderr, "; fastest 50%%:");
		for (int k = 0; k < 7; k++) fprintf(stderr, " %.2f", nl ? ls[k] / nl : 0.0);
		fprintf(stderr, "\n");
		free(lv);
	}
	free(t);
}

/* fused push of every species (pinc_hip_push): kick from E (or none), drift,
 * classification, deposit of the particles that stay into rhoS; positions to
 * xout, velocities in place.  Tiled layout: every sortInterval-th push writes
 * its output in cell order instead (to altX/altV, counting sort on the cell
 * counts of its input), and the push before it counts those cells.  Returns
 * 1 if this push sorted. */
static int push_all(Population *pop, Grid *E, double *const *xout) {
	PincDevPop *dv = pop->dev;
	pinc_geom_t g = dv->geom;
	long n = 1;
	for (int d = 0; d < g.nd; d++) n *= d == g.nd - 1 ? (long)g.nloc + 2 : (long)g.T[d];
	if (dv->rhoN != n) {
		for (int s = 0; s < PINC_MAX_SPECIES; s++) {
			pinc_hip_free(dv->rhoS[s]);
			dv->rhoS[s] = NULL;
		}
		for (int s = 0; s < pop->nSpecies; s++)
			pinc_check(pinc_hip_malloc((void **)&dv->rhoS[s], n * sizeof(double)), "species charge");
		dv->rhoN = n;
	}
	pinc_pop_settle(pop); /* the schedule below reads the last push's counts */
	int sortNow = 0, sortS[PINC_MAX_SPECIES] = {0}, countS[PINC_MAX_SPECIES] = {0};
	int adaptive = dv->sorted && dv->sortFraction > 0;
	dv->keSumsValid = 0;
	g_pinc.errSerial++;
	if (dv->sorted) {
		ensure_keys(pop);
		for (int s = 0; s < pop->nSpecies; s++) {
			if (adaptive) {
				/* sort when this push's input is the one predicted to pass
				 * the displaced fraction (counted by the push before) */
				sortS[s] = dv->sortNext[s];
				const int spreadOk = dv->sortSpread <= 0 || dv->spreadBase[s] <= 0 ||
				                     dv->spreadLast[s] >= dv->sortSpread * dv->spreadBase[s];
				countS[s] = !sortS[s] && ((dv->movedFrac[s] + dv->lastRate[s] >= dv->sortFraction && spreadOk) ||
				                          dv->sinceSort[s] + 1 >= dv->sortMax);
			} else {
				sortS[s] = dv->moves % dv->sortInterval == 0;
				/* (a sorting push never counts: sortInterval 1 recounts) */
				countS[s] = !sortS[s] && (dv->moves + 1) % dv->sortInterval == 0;
			}
			sortNow |= sortS[s];
		}
		dv->moves++;
		/* the in-push sort relies on an input in cell order (its LDS cell
		 * boxes are per block); a population that was never sorted (lattice
		 * order, new particles) gets a sort pass of its own first */
		if (sortNow && !dv->everSorted) sort_tiles(pop);
		dv->everSorted = 1;
	}
	int nd = pop->nDims;
	if (adaptive) {
		/* (spreadCnt follows movedCnt in one block, pinc_pop.c) */
		pinc_check(pinc_hip_memset(dv->movedCnt, 0, 4 * PINC_MAX_SPECIES * sizeof(unsigned long long), g_pinc.stream),
		           "moved counts");
	}
	for (int s = 0; s < pop->nSpecies; s++) {
		int countNext = countS[s];
		pinc_check(pinc_hip_zero(dv->rhoS[s], n, g_pinc.stream), "species charge zero");
		pinc_push_t a;
		memset(&a, 0, sizeof(a));
		if (E) {
			/* every species' rescaled E in one pass over E at the first
			 * species (E does not change during the round) */
			PincDevGrid *eg = E->dev;
			if (eg->scaledAllS < pop->nSpecies) {
				pinc_hip_free(eg->scaledAll);
				pinc_check(pinc_hip_malloc((void **)&eg->scaledAll, (long)pop->nSpecies * eg->n * sizeof(double)),
				           "E scaled");
				eg->scaledAllS = pop->nSpecies;
			}
			if (s == 0)
				pinc_check(pinc_hip_field_chain_all(eg->d, eg->scaledAll, eg->n, dv->qm, dv->mq, 1.0, pop->nSpecies,
				                                    g_pinc.stream),
				           "E chain");
			a.Es = eg->scaledAll + (long)s * eg->n;
			a.kick = 1;
		}
		pinc_pop_t p = pinc_devpop(pop);
		long np = pop->iStop[s] - pop->iStart[s];
		long chunks = dv->chunkBase[s + 1] - dv->chunkBase[s];
		for (int d = 0; d < 3; d++) {
			a.xout[d] = sortNow ? dv->altX[d] : xout[d];
			a.vout[d] = sortNow ? dv->altV[d] : dv->p.v[d];
		}
		a.rhoS = dv->rhoS[s];
		a.thr = g_pinc.thr;
		a.flags = dv->flags;
		a.chunkCount = dv->chunkCount + dv->chunkBase[s];
		a.maxVel = g_pinc.maxVel;
		a.errFlag = g_pinc.dErr;
		a.wrapMask = wrap_mask(pop);
		a.kePartial = dv->kePartial;
		a.tileWidth = dv->tileWidth;
		a.flagsSparse = pinc_flags_before_write(pop, s, 1);
		pinc_check(pinc_hip_memset(a.chunkCount, 0, chunks * sizeof(int), g_pinc.stream), "chunk counts");
		if (adaptive) {
			a.moved = dv->movedCnt + s;
			a.emigTotal = dv->emigCnt + s;
			if (dv->sortSpread > 0 || g_pinc.traceSort) a.spread = dv->spreadCnt + s;
		}
		if (dv->objInside && dv->objHi[0] >= dv->objLo[0]) { /* (empty box: no object node in this slab) */
			a.objInside = dv->objInside;
			a.objSy = dv->objSy;
			a.objSz = dv->objSz;
			a.objNodes = dv->objNodes;
			a.objCount = dv->objCount + (long)s * dv->objK;
			for (int d = 0; d < 3; d++) {
				a.objLo[d] = dv->objLo[d];
				a.objHi[d] = dv->objHi[d];
			}
		}
		if (dv->objCount)
			pinc_check(pinc_hip_memset(dv->objCount + (long)s * dv->objK, 0, dv->objK * sizeof(int), g_pinc.stream),
			           "object counts");
		/* a species left in order by a sorting push still goes to the
		 * alternate arrays (swapped for all species) */
		dv->permId[s] = !sortS[s];
		if (sortS[s]) {
			if (!dv->cntValid[s]) {
				pinc_check(pinc_hip_memset(dv->keyCnt[s], 0, (dv->nKeys + 1) * sizeof(int), g_pinc.stream), "keys");
				pinc_check(pinc_hip_count_keys(p, s, 0, g, dv->tileWidth, dv->keyCnt[s], g_pinc.stream), "count keys");
			}
			pinc_check(pinc_hip_scan_keys(dv->keyCnt[s], dv->nKeys, dv->keyCur[s], dv->keyWork[s], g_pinc.stream),
			           "scan keys");
			a.cursor = dv->keyCur[s];
			dv->cellValid[s] = -1;
		}
		if (countNext) {
			pinc_check(pinc_hip_memset(dv->keyNext[s], 0, (dv->nKeys + 1) * sizeof(int), g_pinc.stream), "keys");
			a.cntNext = dv->keyNext[s];
		}
		int nb = 0;
		unsigned long long *ts = NULL;
		if (g_pinc.traceSort > 1) {
			/* 8 timestamps per push block (pinc_hip_push_chunk particles), then
			 * the diagnostic counters */
			const long nbk = np / pinc_hip_push_chunk() + 1;
			pinc_check(pinc_hip_malloc((void **)&ts, (nbk * 8 + 8) * sizeof(*ts)), "push timestamps");
			pinc_check(pinc_hip_memset(ts + nbk * 8, 0, 8 * sizeof(*ts), g_pinc.stream), "push diagnostics");
			a.tstamp = ts;
			a.diag = ts + nbk * 8;
		}
		const int kind = sortS[s] ? PINC_PROBE_PUSH_SORT : countNext ? PINC_PROBE_PUSH_COUNT : PINC_PROBE_PUSH_PLAIN;
		int slot = E ? pinc_probe_begin(PINC_PROBE_PUSH) : -1;
		pinc_probe_tag(PINC_PROBE_PUSH, slot, s | (sortS[s] ? 2 : countNext ? 1 : 0) << 8);
		int slotK = E ? pinc_probe_begin(kind) : -1;
		pinc_check(pinc_hip_push(p, s, g, &a, &nb, g_pinc.stream), "push");
		if (ts) {
			push_phase_report(ts, a.diag, nb, s, sortS[s], countNext, a.xout, pop->iStart[s], np);
			pinc_hip_free(ts);
		}
		/* pos R+W, vel R+W (32 B per dim per particle) + E R (8 B per value
		 * per node) + rho flush (8 B per node) */
		if (E) {
			const double bytes = 32.0 * nd * np + 8.0 * (nd + 1) * (double)n;
			pinc_probe_end(kind, slotK, bytes);
			pinc_probe_end(PINC_PROBE_PUSH, slot, bytes);
		}
		if (E) {
			/* two-stage (block partials of the partials): deterministic and
			 * fast for a million partials */
			double *keOut = adaptive ? (double *)(dv->spreadCnt + PINC_MAX_SPECIES) + s : PINC_SLOT(16 + s);
			if (nb > 0) pinc_check(pinc_hip_sum(dv->kePartial, nb, g_pinc.dScratch, keOut, g_pinc.stream), "ke");
			else pinc_check(pinc_hip_memset(keOut, 0, sizeof(double), g_pinc.stream), "ke");
		}
		if (countNext) {
			int *t = dv->keyCnt[s];
			dv->keyCnt[s] = dv->keyNext[s];
			dv->keyNext[s] = t;
			dv->cntValid[s] = 1;
		} else if (dv->sorted) {
			dv->cntValid[s] = 0;
		}
	}
	if (adaptive) {
		if (!dv->hostCnt) {
			pinc_check(pinc_hip_host_alloc((void **)&dv->hostCnt, 4 * PINC_MAX_SPECIES * sizeof(unsigned long long)),
			           "counter block");
			pinc_check(pinc_hip_event_create(&dv->cntEvent), "counter block");
		}
		pinc_check(pinc_hip_d2h_async(dv->hostCnt, dv->movedCnt, 4 * PINC_MAX_SPECIES * sizeof(unsigned long long),
		                              g_pinc.stream),
		           "moved, spread and energy readback");
		pinc_check(pinc_hip_event_record(dv->cntEvent, g_pinc.stream), "counter block");
		memcpy(dv->cntSortS, sortS, sizeof(sortS));
		memcpy(dv->cntCountS, countS, sizeof(countS));
		dv->cntE = E != NULL;
		dv->cntPending = 1;
	}
	dv->depValid = 1;
	dv->depExtracted = 0;
	return sortNow;
}

void pinc_pop_settle(Population *pop) {
	PincDevPop *dv = pop->dev;
	if (!dv || !dv->cntPending) return;
	pinc_check(pinc_hip_event_sync(dv->cntEvent), "moved, spread and energy readback");
	dv->cntPending = 0;
	const unsigned long long *cnt = dv->hostCnt;
	const unsigned long long *mv = cnt, *sp = cnt + PINC_MAX_SPECIES;
	const int *sortS = dv->cntSortS, *countS = dv->cntCountS;
	memcpy(dv->emigLast, cnt + 3 * PINC_MAX_SPECIES, sizeof(dv->emigLast));
	dv->emigValid = 1;
	if (dv->cntE) {
		memcpy(dv->keSums, cnt + 2 * PINC_MAX_SPECIES, sizeof(dv->keSums));
		dv->keSumsValid = 1;
		if (dv->keDeferred)
			for (int s = 0; s < pop->nSpecies; s++) pop->kinEnergy[s] = dv->keSums[s] * (0.5 * pop->mass[s]);
	}
	dv->keDeferred = 0;
	for (int s = 0; s < pop->nSpecies; s++) {
		long np = pop->iStop[s] - pop->iStart[s];
		double rate = np > 0 ? (double)mv[s] / (double)np : 0.0;
		/* mean input cell box of this push's blocks */
		const long chunk = pinc_hip_push_chunk();
		const double blocks = (double)((np + chunk - 1) / chunk);
		dv->spreadLast[s] = blocks > 0 ? (double)sp[s] / blocks : 0.0;
		if (sortS[s]) dv->spreadBase[s] = 0;
		if (dv->sinceSort[s] == 1 && !sortS[s]) dv->spreadBase[s] = dv->spreadLast[s];
		dv->movedFrac[s] = sortS[s] ? rate : dv->movedFrac[s] + rate;
		dv->sinceSort[s] = sortS[s] ? 1 : dv->sinceSort[s] + 1;
		dv->lastRate[s] = rate;
		dv->sortNext[s] = countS[s];
		if (g_pinc.traceSort)
			fprintf(stderr, "[pinc] push %ld species %d: moved %.4f, displaced %.4f, cell box %.1f (x%.2f)%s%s\n",
			        dv->moves, s, rate, dv->movedFrac[s], dv->spreadLast[s],
			        dv->spreadBase[s] > 0 ? dv->spreadLast[s] / dv->spreadBase[s] : 0.0, sortS[s] ? ", sorted" : "",
			        countS[s] ? ", counted" : "");
	}
}

/* dst[d] = the kicked velocities of species s pending after a sorting push,
 * in the current particle order (n per component, device).  A species the
 * push left in order has them in altV.  A sorted one gets the kick again:
 * from its unkicked velocities (p.v, which a sorting push only reads), with
 * the push's E and k_accel, whose arithmetic is the fused kick's
 * (puInterp3D1's expression order, no contraction, E read as stored), so
 * the velocities are bit-identical.  This replaces a permutation that every
 * sorting push wrote (4 B per particle) for this rare path (a read or an
 * extract between puAcc and puMove). */
void pinc_pending_vel(const Population *pop, int s, double *const *dst) {
	const PincDevPop *dv = pop->dev;
	long a = pop->iStart[s], n = pop->iStop[s] - a;
	int nd = pop->nDims;
	if (n <= 0) return;
	for (int d = 0; d < nd; d++) {
		const double *src = (dv->permId[s] ? dv->altV[d] : dv->p.v[d]) + a;
		if (dst[d] != src)
			pinc_check(pinc_hip_d2d(dst[d], src, n * sizeof(double), g_pinc.stream), "pending velocities");
	}
	if (dv->permId[s] || dv->vKicked[s]) return;
	if (!dv->pendingE) msg(ERROR, "pending sorted push without its E");
	if (!pinc_grid_live(dv->pendingE, dv->pendingESerial) || dv->pendingE->dev->gen != dv->pendingEGen)
		/* this catches a freed or reallocated E, and a writer that called
		 * pinc_grid_touch without the re-kick above it; a device write that
		 * skips pinc_grid_touch leaves gen as it was and is not seen here, so
		 * every E-writing operator must call it (pinc_grid.c) */
		msg(ERROR, "internal: E was freed, reallocated or touched between puAcc and a re-kick of the pending "
		           "sorting push");
	PincDevGrid *eg = dv->pendingE->dev;
	/* species s's rescaled E of the push round (E unchanged since: checked
	 * above), else made here */
	const double *es = eg->scaledAll && s < eg->scaledAllS ? eg->scaledAll + (long)s * eg->n : NULL;
	if (!es) {
		if (!eg->scaled) pinc_check(pinc_hip_malloc((void **)&eg->scaled, eg->n * sizeof(double)), "E scaled");
		pinc_check(pinc_hip_field_chain(eg->d, eg->scaled, eg->n, dv->qm, dv->mq, 1.0, s, g_pinc.stream), "E chain");
		es = eg->scaled;
	}
	pinc_pop_t p = pinc_devpop(pop);
	/* (species s only is touched: indices iStart[s] .. iStop[s] - 1) */
	for (int d = 0; d < nd; d++) p.v[d] = dst[d] - a;
	int nb = 0;
	pinc_check(pinc_hip_accelerate(p, s, eg->geom, es, dv->kePartial, &nb, g_pinc.stream), "pending kick");
}

/* The populations with a pending fused push (main.c has one).  Before a
 * grid is written, a pending sorting push that kicked with it re-applies its
 * kick to the unkicked velocities in place (p.v, in the current order), so
 * that a later read or a dropped move does not need that E any more: main.c's
 * initial half step rescales E right after puAcc (gMul(E, 2), main.c:183-185),
 * and a read of the population after it must see the half kick. */
static Population *g_pendPop[8];

void pinc_pending_register(Population *pop) {
	for (int i = 0; i < 8; i++)
		if (g_pendPop[i] == pop) return;
	for (int i = 0; i < 8; i++)
		if (!g_pendPop[i]) {
			g_pendPop[i] = pop;
			return;
		}
	msg(ERROR, "more than 8 populations with pending pushes");
}

void pinc_pending_unregister(Population *pop) {
	for (int i = 0; i < 8; i++)
		if (g_pendPop[i] == pop) g_pendPop[i] = NULL;
}

void pinc_grid_touch(Grid *g) {
	for (int i = 0; i < 8; i++) {
		Population *pop = g_pendPop[i];
		if (!pop) continue;
		PincDevPop *dv = pop->dev;
		if (!dv->pending || !dv->pendingSorted || dv->pendingE != g) continue;
		for (int s = 0; s < pop->nSpecies; s++) {
			if (dv->permId[s] || dv->vKicked[s]) continue;
			double *dst[3] = {NULL, NULL, NULL};
			for (int d = 0; d < pop->nDims; d++) dst[d] = dv->p.v[d] + pop->iStart[s];
			pinc_pending_vel(pop, s, dst);
			dv->vKicked[s] = 1;
		}
	}
	g->dev->gen++;
}

static void swap_pos(PincDevPop *dv, int nd, int vel) {
	for (int d = 0; d < nd; d++) {
		double *t = dv->p.x[d];
		dv->p.x[d] = dv->altX[d];
		dv->altX[d] = t;
		if (vel) {
			t = dv->p.v[d];
			dv->p.v[d] = dv->altV[d];
			dv->altV[d] = t;
		}
	}
}

static void classify(Population *pop, int doMove) {
	pinc_pop_flush_host(pop);
	pinc_pop_settle(pop); /* (before emigValid changes below) */
	if (!g_pinc.thrSet) msg(ERROR, "gCreateNeighborhood must run before puMove/extract");
	PincDevPop *dv = pop->dev;
	int nd = pop->nDims;
	if (!doMove && dv->pending) {
		/* flags recomputed for the current positions: drop the pending move
		 * (a sorted one first puts the kicked velocities back in order) */
		if (dv->pendingSorted)
			for (int s = 0; s < pop->nSpecies; s++) {
				double *dst[3];
				for (int d = 0; d < 3; d++) dst[d] = d < nd ? dv->p.v[d] + pop->iStart[s] : NULL;
				pinc_pending_vel(pop, s, dst);
			}
		dv->pending = dv->pendingSorted = 0;
		/* its object counts go with it */
		if (dv->objCount)
			pinc_check(pinc_hip_memset(dv->objCount, 0, (long)PINC_MAX_SPECIES * dv->objK * sizeof(int), g_pinc.stream),
			           "object counts");
	}
	if (doMove && dv->pending) {
		/* the fused puAcc already moved, classified and deposited */
		swap_pos(dv, nd, dv->pendingSorted);
		dv->pending = dv->pendingSorted = 0;
		dv->flagsValid = 1;
		dv->depValid = 1;
		dv->depExtracted = 0;
		return;
	}
	if (doMove && !dv->sorted) maybe_sort(pop);
	if (doMove && dv->fused) {
		if (push_all(pop, NULL, dv->p.x)) swap_pos(dv, nd, 1);
		dv->flagsValid = 1;
		return;
	}
	for (int s = 0; s < PINC_MAX_SPECIES; s++) dv->cntValid[s] = 0;
	dv->depValid = 0;
	dv->emigValid = 0; /* (flags of this classification: not counted) */
	/* every launch gets dErr: a classification without a move still sets the
	 * out-of-frame bit, so the next assert read must not be skipped */
	g_pinc.errSerial++;
	int wrapMask = wrap_mask(pop);
	pinc_pop_t p = pinc_devpop(pop);
	for (int s = 0; s < pop->nSpecies; s++) {
		long n = pop->iStop[s] - pop->iStart[s];
		int slot = doMove ? pinc_probe_begin(PINC_PROBE_MOVE) : -1;
		pinc_flags_before_write(pop, s, 0);
		pinc_check(pinc_hip_move_classify(p, s, doMove, g_pinc.thr, dv->flags, dv->chunkCount + dv->chunkBase[s],
		                                  g_pinc.maxVel, g_pinc.dErr, wrapMask, g_pinc.stream),
		           "move/classify");
		/* read pos+vel, write pos: 72 B per 3-D particle */
		pinc_probe_end(PINC_PROBE_MOVE, slot, 24.0 * pop->nDims * n);
	}
	dv->flagsValid = 1;
}

void puMove(Population *pop, Object *obj) {
	(void)obj; /* particle-object collisions are out of scope (fact 6) */
	/* a pending fused move is a pointer swap: no device work, no timer
	 * events (each costs the host an event record while the GPU waits) */
	const int timed = !pop->dev->pending || pop->dev->hostDirty;
	if (timed) pinc_phase_begin(0);
	classify(pop, 1);
	if (timed) pinc_phase_end(0);
}

/* ------------------------------------------------------------- extract -- */
static void extract(Population *pop, MpiInfo *m) {
	pinc_pop_flush_host(pop);
	PincDevPop *dv = pop->dev;
	pinc_pop_settle(pop);
	/* the flags of the last push, whose flagged counts are known */
	const int known = g_pinc.extractSkip && dv->flagsValid && dv->emigValid;
	if (!dv->flagsValid) classify(pop, 0);
	int ns = pop->nSpecies, nN = m->nNeighbors;
	int work = !known;
	for (int s = 0; s < ns; s++) work |= dv->emigLast[s] != 0;
	if (work) pinc_phase_begin(1);
	memset(m->nEmigrants, 0, nN * ns * sizeof(long));
	for (int s = 0; s < ns; s++) {
		if (known && dv->emigLast[s] == 0) {
			/* nothing flagged to leave: the extraction would find nothing
			 * (and every flag of the last write is the centre) */
			if (dv->flagState[s] == PINC_FLAGS_PENDING) dv->flagState[s] = PINC_FLAGS_CLEAN;
			dv->nEmig[s] = 0;
			memset(dv->neCount[s], 0, sizeof(dv->neCount[s]));
			if (dv->depValid) dv->depEnd[s] = pop->iStop[s];
			continue;
		}
		for (int attempt = 0;; attempt++) {
			pinc_pop_t p = pinc_devpop(pop);
			long nEmig = 0;
			int rc = pinc_hip_extract(p, s, dv->flags, dv->chunkCount + dv->chunkBase[s], m->neighborhoodCenter, nN,
			                          dv->ws[s], &nEmig, dv->neCount[s], g_pinc.stream);
			if (rc == PINC_ERR_CAPACITY && attempt == 0) {
				pinc_pop_grow_ws(pop, s, nEmig);
				continue;
			}
			pinc_check(rc, "extract emigrants");
			pinc_flags_after_extract(pop, s, p.iStop[s] - p.iStart[s]);
			dv->nEmig[s] = nEmig;
			break;
		}
		pop->iStop[s] -= dv->nEmig[s];
		/* particles the fused push collected into an object are extracted
		 * last (PINC_NE_SINK) and not migrated */
		dv->nEmig[s] -= dv->neCount[s][PINC_NE_SINK];
		if (dv->depValid) dv->depEnd[s] = pop->iStop[s];
		if (dv->tiled && dv->cellValid[s] > pop->iStop[s] - pop->iStart[s])
			dv->cellValid[s] = pop->iStop[s] - pop->iStart[s];
		for (int ne = 0; ne < nN; ne++) m->nEmigrants[ne * ns + s] = dv->neCount[s][ne];
	}
	dv->flagsValid = 0;
	dv->emigValid = 0;
	if (dv->depValid) dv->depExtracted = 1;
	if (work) pinc_phase_end(1);
}

void puExtractEmigrants3D(Population *pop, MpiInfo *m) { extract(pop, m); }
void puExtractEmigrantsND(Population *pop, MpiInfo *m) { extract(pop, m); }

/* ------------------------------------------------------------- migrate -- */
/* (re)allocate a pair of record buffers to hold at least `need` records */
static void ensure_pair(double **buf, long *cap, long need) {
	if (need <= *cap && buf[0]) return;
	pinc_check(pinc_hip_stream_sync(g_pinc.stream), "buf sync");
	long c = need + need / 4 + 1024;
	for (int k = 0; k < 2; k++) {
		pinc_hip_free(buf[k]);
		pinc_check(pinc_hip_malloc((void **)&buf[k], c * PINC_REC * sizeof(double)), "migrant buffer");
	}
	*cap = c;
}

static void puMigrateImport(Population *pop, MpiInfo *m) {
	PincDevPop *dv = pop->dev;
	int ns = pop->nSpecies, nd = pop->nDims;
	pinc_geom_t g = dv->geom;
	int T[3] = {1, 1, 1};
	for (int d = 0; d < nd; d++) T[d] = d == nd - 1 ? g.nloc : g.T[d];
	int P3 = pinc_ipow3(nd - 1);
	if (g_pinc.nranks == 1) {
		/* every neighbour is this rank: messages arrive in the order they
		 * were sent (by direction ne), each shifted by its receive tag */
		for (int s = 0; s < ns; s++) {
			long E = dv->nEmig[s];
			pinc_pop_t p = pinc_devpop(pop);
			pinc_check(pinc_hip_import(p, s, pop->iStop[s] - pop->iStart[s], dv->ws[s].buf, dv->ws[s].cap,
			                           dv->ws[s].bufNe, 0, E, T, (1 << nd) - 1, g_pinc.stream),
			           "import");
			pop->iStop[s] += E;
			for (int ne = 0; ne < m->nNeighbors; ne++)
				m->nImmigrants[puNeighborToReciprocal(ne, nd) * ns + s] = dv->neCount[s][ne];
		}
		dv->flagsValid = 0;
		return;
	}
	/* slab decomposition: directions whose slab digit is 0 go down, 2 go up,
	 * 1 stay.  The buffer of each species is sorted by direction, so these
	 * are three contiguous segments. */
	long nDown[PINC_MAX_SPECIES], nLocal[PINC_MAX_SPECIES], nUp[PINC_MAX_SPECIES];
	long totDown = 0, totUp = 0;
	for (int s = 0; s < ns; s++) {
		nDown[s] = nLocal[s] = nUp[s] = 0;
		for (int ne = 0; ne < m->nNeighbors; ne++) {
			int dig = ne / P3;
			long c = dv->neCount[s][ne];
			if (dig == 0) nDown[s] += c;
			else if (dig == 1) nLocal[s] += c;
			else nUp[s] += c;
		}
		totDown += nDown[s];
		totUp += nUp[s];
	}
	/* exchange counts (exchangeNMigrants, pusher.c:914-938) */
	int P = g_pinc.nranks, r = g_pinc.rank;
	int up = (r + 1) % P, dn = (r - 1 + P) % P;
	double cnt[4 * PINC_MAX_SPECIES];
	for (int s = 0; s < ns; s++) {
		cnt[s] = (double)nUp[s];
		cnt[PINC_MAX_SPECIES + s] = (double)nDown[s];
	}
	double *dc = PINC_SLOT(64);
	pinc_check(pinc_hip_h2d(dc, cnt, 2 * PINC_MAX_SPECIES * sizeof(double), g_pinc.stream), "counts");
	{
		int sp[2] = {up, dn}, rp[2] = {dn, up};
		void *sb[2] = {dc, dc + PINC_MAX_SPECIES};
		void *rb[2] = {dc + 2 * PINC_MAX_SPECIES, dc + 3 * PINC_MAX_SPECIES};
		long nb[2] = {ns * sizeof(double), ns * sizeof(double)};
		pinc_comm_exchange(2, sp, sb, nb, rp, rb, nb, "count exchange");
	}
	pinc_check(pinc_hip_d2h(cnt, dc, 4 * PINC_MAX_SPECIES * sizeof(double), g_pinc.stream), "counts");
	long fromDown[PINC_MAX_SPECIES], fromUp[PINC_MAX_SPECIES], totFromDown = 0, totFromUp = 0;
	for (int s = 0; s < ns; s++) {
		fromDown[s] = (long)cnt[2 * PINC_MAX_SPECIES + s];
		fromUp[s] = (long)cnt[3 * PINC_MAX_SPECIES + s];
		totFromDown += fromDown[s];
		totFromUp += fromUp[s];
	}
	/* pack payloads: records of all species back to back */
	ensure_pair(dv->sendBuf, &dv->sendCap, totUp > totDown ? totUp : totDown);
	ensure_pair(dv->recvBuf, &dv->recvCap, totFromUp > totFromDown ? totFromUp : totFromDown);
	long oUp = 0, oDown = 0;
	for (int s = 0; s < ns; s++) {
		pinc_extract_ws_t *w = &dv->ws[s];
		pinc_check(pinc_hip_pack(w->buf, w->cap, w->bufNe, nDown[s] + nLocal[s], nUp[s], nd,
		                         dv->sendBuf[0] + oUp * PINC_REC, g_pinc.stream), "pack up");
		pinc_check(pinc_hip_pack(w->buf, w->cap, w->bufNe, 0, nDown[s], nd, dv->sendBuf[1] + oDown * PINC_REC,
		                         g_pinc.stream), "pack down");
		oUp += nUp[s];
		oDown += nDown[s];
	}
	{
		int sp[2] = {up, dn}, rp[2] = {dn, up};
		void *sb[2] = {dv->sendBuf[0], dv->sendBuf[1]};
		void *rb[2] = {dv->recvBuf[0], dv->recvBuf[1]};
		long snb[2] = {totUp * PINC_REC * (long)sizeof(double), totDown * PINC_REC * (long)sizeof(double)};
		long rnb[2] = {totFromDown * PINC_REC * (long)sizeof(double), totFromUp * PINC_REC * (long)sizeof(double)};
		pinc_comm_exchange(2, sp, sb, snb, rp, rb, rnb, "migrant exchange");
	}
	/* import in receive-tag order 26..0: from above, then local, then from below */
	long offUp = 0, offDown = 0;
	for (int s = 0; s < ns; s++) {
		pinc_pop_t p = pinc_devpop(pop);
		long dst = pop->iStop[s] - pop->iStart[s];
		if (dst + fromUp[s] + nLocal[s] + fromDown[s] > pop->iStart[s + 1] - pop->iStart[s])
			msg(ERROR, "population overflow on migration (species %d): raise population:nAlloc", s);
		pinc_check(pinc_hip_import_rec(p, s, dst, dv->recvBuf[1] + offUp * PINC_REC, fromUp[s], T, g_pinc.stream),
		           "import from above");
		dst += fromUp[s];
		pinc_check(pinc_hip_import(p, s, dst, dv->ws[s].buf, dv->ws[s].cap, dv->ws[s].bufNe, nDown[s], nLocal[s], T,
		                           (1 << nd) - 1, g_pinc.stream),
		           "import local");
		dst += nLocal[s];
		pinc_check(pinc_hip_import_rec(p, s, dst, dv->recvBuf[0] + offDown * PINC_REC, fromDown[s], T,
		                               g_pinc.stream),
		           "import from below");
		dst += fromDown[s];
		pop->iStop[s] = pop->iStart[s] + dst;
		offUp += fromUp[s];
		offDown += fromDown[s];
	}
	dv->flagsValid = 0;
	
}

void puMigrate(Population *pop, MpiInfo *m, Grid *grid) {
	(void)grid;
	pinc_pop_flush_host(pop);
	PincDevPop *dv = pop->dev;
	int ns = pop->nSpecies;
	/* one rank without emigrants: nothing to import (no timer events) */
	int work = g_pinc.nranks > 1;
	for (int s = 0; s < ns; s++) work |= dv->nEmig[s] != 0;
	if (work) pinc_phase_begin(2);
	memset(m->nImmigrants, 0, m->nNeighbors * ns * sizeof(long));
	long before[PINC_MAX_SPECIES];
	for (int s = 0; s < ns; s++) before[s] = pop->iStop[s] - pop->iStart[s];
	puMigrateImport(pop, m);
	/* sorted layout: the imported particles join the key counts */
	if (dv->sorted)
		for (int s = 0; s < ns; s++)
			if (dv->cntValid[s] && pop->iStop[s] - pop->iStart[s] > before[s]) {
				pinc_pop_t p = pinc_devpop(pop);
				pinc_check(pinc_hip_count_keys(p, s, before[s], dv->geom, dv->tileWidth, dv->keyCnt[s], g_pinc.stream),
				           "count immigrant keys");
			}
	if (work) pinc_phase_end(2);
}

/* ------------------------------------------------------------- deposit -- */
/* gZero; per species gMul(1/q), scatter, gMul(q) (pusher.c:512-572): the
 * consecutive gMul(q_{s-1}), gMul(1/q_s) become one two-rounding pass. */
static void distr(const Population *pop, Grid *rho) {
	pinc_pop_flush_host(pop);
	pinc_phase_begin(3);
	PincDevGrid *g = rho->dev;
	g->depPop = pop;
	g->depOrder = 1;
	g->folds = 0;
	PincDevPop *dvp = pop->dev;
	if (dvp->depValid && dvp->depExtracted && dvp->rhoN == g->n) {
		/* fused push: the particles that stayed are in rhoS; add the ones
		 * imported since (the tail of each species), then combine */
		for (int s = 0; s < pop->nSpecies; s++) {
			if (pop->iStop[s] <= dvp->depEnd[s]) continue;
			pinc_pop_t t = pinc_devpop(pop);
			t.iStart[s] = dvp->depEnd[s];
			pinc_check(pinc_hip_deposit(t, s, g->geom, dvp->rhoS[s], g_pinc.stream), "deposit (immigrants)");
		}
		pinc_check(pinc_hip_rho_combine(g->d, (const double *const *)dvp->rhoS, pop->charge, pop->nSpecies, g->n,
		                                g_pinc.stream),
		           "rho combine");
		dvp->depValid = dvp->depExtracted = 0;
		g->ghostsValid = 0;
		pinc_phase_end(3);
		return;
	}
	pinc_check(pinc_hip_zero(g->d, g->n, g_pinc.stream), "distr zero");
	pinc_pop_t p = pinc_devpop(pop);
	for (int s = 0; s < pop->nSpecies; s++) {
		if (s > 0)
			pinc_check(pinc_hip_scale2(g->d, g->n, pop->charge[s - 1], 1.0 / pop->charge[s], g_pinc.stream),
			           "distr scale");
		int slot = pinc_probe_begin(PINC_PROBE_DEPOSIT);
		PincDevPop *dv = pop->dev;
		if (dv->tiled && dv->cellValid[s] >= 0)
			pinc_check(pinc_hip_deposit_cells(p, s, g->geom, dv->tileWidth, dv->sortWork[s] + (dv->sortKeys + 1),
			                                  dv->cellValid[s], g->d, g_pinc.stream),
			           "deposit (cells)");
		else
			pinc_check(pinc_hip_deposit(p, s, g->geom, g->d, g_pinc.stream), "deposit");
		/* read pos (8 B per dim per particle) + write rho (8 B per node) */
		pinc_probe_end(PINC_PROBE_DEPOSIT, slot,
		               8.0 * pop->nDims * (pop->iStop[s] - pop->iStart[s]) + 8.0 * g->n);
	}
	pinc_check(pinc_hip_scale(g->d, g->n, pop->charge[pop->nSpecies - 1], g_pinc.stream), "distr scale");
	g->ghostsValid = 0;
	pinc_phase_end(3);
}

/* gZero; per species gMul(1/q), one unit per particle at its nearest node,
 * gMul(q) (puDistrND0, pusher.c:640-668).  A fused push's CIC deposit is not
 * used. */
void puDistrND0(const Population *pop, Grid *rho) {
	pinc_pop_flush_host(pop);
	pinc_phase_begin(3);
	PincDevGrid *g = rho->dev;
	g->depPop = pop;
	g->depOrder = 0;
	g->folds = 0;
	pop->dev->depValid = pop->dev->depExtracted = 0;
	pinc_check(pinc_hip_zero(g->d, g->n, g_pinc.stream), "distr zero");
	pinc_pop_t p = pinc_devpop(pop);
	for (int s = 0; s < pop->nSpecies; s++) {
		if (s > 0)
			pinc_check(pinc_hip_scale2(g->d, g->n, pop->charge[s - 1], 1.0 / pop->charge[s], g_pinc.stream),
			           "distr scale");
		pinc_check(pinc_hip_deposit_ngp(p, s, g->geom, g->d, g_pinc.stream), "deposit (NGP)");
	}
	pinc_check(pinc_hip_scale(g->d, g->n, pop->charge[pop->nSpecies - 1], g_pinc.stream), "distr scale");
	g->ghostsValid = 0;
	pinc_phase_end(3);
}

/* main.c:226 and :232 both call gHaloOp(addSlice, rho, FROMHALO) on one
 * deposit; ghost values are not cleared in between, so a
 * weight on a node with g ghost coordinates counts 2^g times.  Slab ghost
 * planes are stored and folded again by the second call; the non-slab
 * dimensions were wrapped at deposit.  Before that second fold, add the
 * weight the plain deposit did not carry (geom.literal = 2,
 * literal_node_factor in k_particles.hip), with the species chain of the
 * deposit. */
void pinc_literal_second_fold(const Population *pop, Grid *rho, int order) {
	PincDevGrid *g = rho->dev;
	pinc_geom_t geo = g->geom;
	geo.literal = 2;
	if (!g->lit) pinc_check(pinc_hip_malloc((void **)&g->lit, g->n * sizeof(double)), "second fold scratch");
	pinc_check(pinc_hip_zero(g->lit, g->n, g_pinc.stream), "second fold");
	pinc_pop_t p = pinc_devpop(pop);
	for (int s = 0; s < pop->nSpecies; s++) {
		if (s > 0)
			pinc_check(pinc_hip_scale2(g->lit, g->n, pop->charge[s - 1], 1.0 / pop->charge[s], g_pinc.stream),
			           "second fold scale");
		if (order == 0) pinc_check(pinc_hip_deposit_ngp(p, s, geo, g->lit, g_pinc.stream), "second fold (NGP)");
		else pinc_check(pinc_hip_deposit(p, s, geo, g->lit, g_pinc.stream), "second fold");
	}
	pinc_check(pinc_hip_scale(g->lit, g->n, pop->charge[pop->nSpecies - 1], g_pinc.stream), "second fold scale");
	pinc_check(pinc_hip_add(g->d, g->lit, g->n, g_pinc.stream), "second fold add");
}

void puDistr3D1(const Population *pop, Grid *rho) { distr(pop, rho); }
void puDistrND1(const Population *pop, Grid *rho) { distr(pop, rho); }

/* ----------------------------------------------------------- accelerate -- */
static void acc(Population *pop, Grid *E, int ke) {
	pinc_pop_flush_host(pop);
	pinc_phase_begin(6);
	PincDevPop *dv = pop->dev;
	if (dv->fused) {
		/* kick now; the drift of the next puMove, its classification and its
		 * deposit ride along (positions to altX, swapped in by puMove) */
		if (!dv->sorted) maybe_sort(pop);
		dv->pending = 0;
		dv->pendingSorted = push_all(pop, E, dv->altX);
		for (int s = 0; s < PINC_MAX_SPECIES; s++) dv->vKicked[s] = 0;
		pinc_pending_register(pop);
		dv->pending = 1;
		dv->pendingE = E;
		dv->pendingESerial = E->dev->serial;
		dv->pendingEGen = E->dev->gen;
		dv->flagsValid = 0;
		if (ke && dv->cntPending) {
			/* the sums come with the sort counters (push_all): kinEnergy is
			 * filled when they are taken in (pinc_pop_settle: pSumKinEnergy,
			 * pWriteEnergy, the next push or extraction) */
			dv->keDeferred = 1;
		} else if (ke) {
			double sums[PINC_MAX_SPECIES];
			pinc_check(pinc_hip_d2h(sums, PINC_SLOT(16), pop->nSpecies * sizeof(double), g_pinc.stream), "ke readback");
			for (int s = 0; s < pop->nSpecies; s++) pop->kinEnergy[s] = sums[s] * (0.5 * pop->mass[s]);
		}
		pinc_phase_end(6);
		return;
	}
	pinc_pop_t p = pinc_devpop(pop);
	int ns = pop->nSpecies;
	for (int s = 0; s < ns; s++) {
		int nb = 0;
		PincDevGrid *eg = E->dev;
		if (!eg->scaled)
			pinc_check(pinc_hip_malloc((void **)&eg->scaled, eg->n * sizeof(double)), "E scaled");
		pinc_check(pinc_hip_field_chain(eg->d, eg->scaled, eg->n, dv->qm, dv->mq, 1.0, s, g_pinc.stream),
		           "E chain");
		int slot = pinc_probe_begin(PINC_PROBE_ACCEL);
		pinc_check(pinc_hip_accelerate(p, s, eg->geom, eg->scaled, dv->kePartial, &nb, g_pinc.stream),
		           "accelerate");
		/* read pos+vel, write vel (72 B per 3-D particle) + read E once */
		pinc_probe_end(PINC_PROBE_ACCEL, slot,
		               24.0 * pop->nDims * (pop->iStop[s] - pop->iStart[s]) + 8.0 * E->dev->n);
		if (nb > 0) pinc_check(pinc_hip_sum(dv->kePartial, nb, g_pinc.dScratch, PINC_SLOT(16 + s), g_pinc.stream), "ke");
		else pinc_check(pinc_hip_memset(PINC_SLOT(16 + s), 0, sizeof(double), g_pinc.stream), "ke");
	}
	if (ke) {
		double sums[PINC_MAX_SPECIES];
		pinc_check(pinc_hip_d2h(sums, PINC_SLOT(16), ns * sizeof(double), g_pinc.stream), "ke readback");
		for (int s = 0; s < ns; s++) pop->kinEnergy[s] = sums[s] * (0.5 * pop->mass[s]);
	}
	pinc_phase_end(6);
}

/* per species: E as rescaled for s, half kick, rotation, half kick, KE */
static void boris(Population *pop, Grid *E, const double *T, const double *S, int ke) {
	pinc_pop_flush_host(pop);
	pinc_phase_begin(6);
	PincDevPop *dv = pop->dev;
	if (dv->pending) msg(ERROR, "Boris push after a fused puAcc without its puMove");
	pinc_pop_t p = pinc_devpop(pop);
	int ns = pop->nSpecies;
	for (int s = 0; s < ns; s++) {
		int nb = 0;
		PincDevGrid *eg = E->dev;
		if (!eg->scaled)
			pinc_check(pinc_hip_malloc((void **)&eg->scaled, eg->n * sizeof(double)), "E scaled");
		pinc_check(pinc_hip_field_chain(eg->d, eg->scaled, eg->n, dv->qm, dv->mq, 1.0, s, g_pinc.stream),
		           "E chain");
		int slot = pinc_probe_begin(PINC_PROBE_ACCEL);
		pinc_check(pinc_hip_boris(p, s, eg->geom, eg->scaled, T + 3 * s, S + 3 * s, dv->kePartial, &nb,
		                          g_pinc.stream),
		           "boris");
		pinc_probe_end(PINC_PROBE_ACCEL, slot,
		               24.0 * pop->nDims * (pop->iStop[s] - pop->iStart[s]) + 8.0 * E->dev->n);
		if (nb > 0) pinc_check(pinc_hip_sum(dv->kePartial, nb, g_pinc.dScratch, PINC_SLOT(16 + s), g_pinc.stream), "ke");
		else pinc_check(pinc_hip_memset(PINC_SLOT(16 + s), 0, sizeof(double), g_pinc.stream), "ke");
	}
	if (ke) {
		double sums[PINC_MAX_SPECIES];
		pinc_check(pinc_hip_d2h(sums, PINC_SLOT(16), ns * sizeof(double), g_pinc.stream), "ke readback");
		for (int s = 0; s < ns; s++) pop->kinEnergy[s] = sums[s] * (0.5 * pop->mass[s]);
	}
	pinc_phase_end(6);
}

void puBoris3D1(Population *pop, Grid *E, const double *T, const double *S) { boris(pop, E, T, S, 0); }
void puBoris3D1KE(Population *pop, Grid *E, const double *T, const double *S) { boris(pop, E, T, S, 1); }

/* puAccND0KE (pusher.c:310-353): per species E as rescaled for it, v += E at
 * the nearest node, KE.  Not fused: the next puMove moves on its own. */
void puAccND0KE(Population *pop, Grid *E) {
	pinc_pop_flush_host(pop);
	pinc_phase_begin(6);
	PincDevPop *dv = pop->dev;
	if (dv->pending) msg(ERROR, "puAccND0KE after a fused puAcc without its puMove");
	pinc_pop_t p = pinc_devpop(pop);
	int ns = pop->nSpecies;
	PincDevGrid *eg = E->dev;
	if (!eg->scaled) pinc_check(pinc_hip_malloc((void **)&eg->scaled, eg->n * sizeof(double)), "E scaled");
	for (int s = 0; s < ns; s++) {
		int nb = 0;
		pinc_check(pinc_hip_field_chain(eg->d, eg->scaled, eg->n, dv->qm, dv->mq, 1.0, s, g_pinc.stream), "E chain");
		pinc_check(pinc_hip_accelerate_ngp(p, s, eg->geom, eg->scaled, dv->kePartial, &nb, g_pinc.stream),
		           "accelerate (NGP)");
		if (nb > 0) pinc_check(pinc_hip_sum(dv->kePartial, nb, g_pinc.dScratch, PINC_SLOT(16 + s), g_pinc.stream), "ke");
		else pinc_check(pinc_hip_memset(PINC_SLOT(16 + s), 0, sizeof(double), g_pinc.stream), "ke");
	}
	double sums[PINC_MAX_SPECIES];
	pinc_check(pinc_hip_d2h(sums, PINC_SLOT(16), ns * sizeof(double), g_pinc.stream), "ke readback");
	for (int s = 0; s < ns; s++) pop->kinEnergy[s] = sums[s] * (0.5 * pop->mass[s]);
	pinc_phase_end(6);
}

void puAcc3D1(Population *pop, Grid *E) { acc(pop, E, 0); }
void puAcc3D1KE(Population *pop, Grid *E) { acc(pop, E, 1); }
void puAccND1(Population *pop, Grid *E) { acc(pop, E, 0); }
void puAccND1KE(Population *pop, Grid *E) { acc(pop, E, 1); }
