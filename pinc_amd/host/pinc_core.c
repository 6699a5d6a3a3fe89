/*
 * pinc_core.c -- io, ini dictionary, method selection, normalisation and the
 * per-process device context of the MI355X PINC hot path (host side, C).
 *
 *   msg / select / ini*   io.c:115-560 (iniparser 3.1 line grammar,
 *                         iniparser.c:555-613; lists io.c:741-841)
 *   uAlloc / uNormalize   units.c:61-252
 *   context               replaces MPI_COMM_WORLD: one HIP stream, one RCCL
 *                         communicator and a device scratch area per process
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <ctype.h>
#include <math.h>
#include <stdarg.h>

PincCtx g_pinc;

/* ---------------------------------------------------------------- msg -- */
static char g_lastError[1024];

/* rank 0 prints (io.c:170-217); before the world is set up (gAllocMpi) the
 * rank comes from the launcher's environment, as MPI_Init has it in main() */
static int msg_rank(void) {
	if (g_pinc.initialised) return g_pinc.rank;
	int r, n, l;
	pinc_launcher_env(&r, &n, &l);
	return r;
}

void msg(msgKind kind, const char *format, ...) {
	char buf[1024];
	va_list ap;
	va_start(ap, format);
	vsnprintf(buf, sizeof(buf), format, ap);
	va_end(ap);
	const char *prefix = "STATUS";
	FILE *stream = stdout;
	switch (kind & 0x0F) {
	case WARNING: prefix = "WARNING"; stream = stderr; break;
	case ERROR: prefix = "ERROR"; stream = stderr; break;
	case TIMER: prefix = "TIMER"; break;
	default: break;
	}
	if ((kind & 0x0F) == ERROR) snprintf(g_lastError, sizeof(g_lastError), "%s", buf);
	if ((kind & ALL) || msg_rank() == 0) {
		/* STATUS lines print as in the reference (only regular() emits them);
		 * PINC_QUIET silences them */
		if ((kind & 0x0F) != STATUS || !getenv("PINC_QUIET")) fprintf(stream, "%s: %s\n", prefix, buf);
		fflush(stream);
	}
	if ((kind & 0x0F) == ERROR) exit(EXIT_FAILURE);
}

const char *pinc_last_error(void) { return g_lastError; }

void pinc_check(int rc, const char *where) {
	if (rc) msg(ERROR, "%s failed: %s", where, pinc_hip_error_string());
}

int pinc_ipow3(int d) {
	int r = 1;
	while (d--) r *= 3;
	return r;
}

/* ---------------------------------------------------------- dictionary -- */
typedef struct { char *key, *val; } Entry;
struct dictionary { Entry *e; int n, cap; };

static char *dupstr(const char *s) {
	size_t n = strlen(s);
	char *r = malloc(n + 1);
	memcpy(r, s, n + 1);
	return r;
}

static void lowercase(char *s) {
	for (; *s; s++) *s = (char)tolower((unsigned char)*s);
}

static char *trim(char *s) {
	while (*s && isspace((unsigned char)*s)) s++;
	char *e = s + strlen(s);
	while (e > s && isspace((unsigned char)e[-1])) e--;
	*e = '\0';
	return s;
}

void iniSet(dictionary *ini, const char *key, const char *value) {
	char *k = dupstr(key);
	lowercase(k);
	for (int i = 0; i < ini->n; i++) {
		if (!strcmp(ini->e[i].key, k)) {
			free(ini->e[i].val);
			ini->e[i].val = dupstr(value);
			free(k);
			return;
		}
	}
	if (ini->n == ini->cap) {
		ini->cap = ini->cap ? 2 * ini->cap : 64;
		ini->e = realloc(ini->e, ini->cap * sizeof(Entry));
	}
	ini->e[ini->n].key = k;
	ini->e[ini->n].val = dupstr(value);
	ini->n++;
}

static void parseLine(dictionary *ini, char *raw, char *section) {
	char *line = trim(raw);
	size_t len = strlen(line);
	if (!len || line[0] == '#' || line[0] == ';') return;
	if (line[0] == '[' && line[len - 1] == ']') {
		line[len - 1] = '\0';
		strcpy(section, trim(line + 1));
		lowercase(section);
		return;
	}
	char *eq = strchr(line, '=');
	if (!eq) return;
	*eq = '\0';
	char *key = trim(line), *val = trim(eq + 1);
	if (val[0] == '"' || val[0] == '\'') {
		char *end = strchr(val + 1, val[0]);
		if (end) {
			*end = '\0';
			val++;
		}
	} else {
		char *c = strpbrk(val, ";#");
		if (c) *c = '\0';
		val = trim(val);
	}
	char full[512];
	snprintf(full, sizeof(full), "%s:%s", section, key);
	iniSet(ini, full, val);
}

dictionary *iniFromString(const char *text) {
	dictionary *ini = calloc(1, sizeof(*ini));
	char section[256] = "";
	char *copy = dupstr(text), *save = NULL;
	for (char *ln = strtok_r(copy, "\n", &save); ln; ln = strtok_r(NULL, "\n", &save))
		parseLine(ini, ln, section);
	free(copy);
	return ini;
}

/* argv[1] = ini file, then key=value overrides (io.c:254-311) */
dictionary *iniOpen(int argc, char *argv[]) {
	if (argc < 2) msg(ERROR, "at least one argument expected (the input file).");
	FILE *f = fopen(argv[1], "rb");
	if (!f) msg(ERROR, "Failed to open %s.", argv[1]);
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	fseek(f, 0, SEEK_SET);
	char *buf = malloc(n + 1);
	if (fread(buf, 1, n, f) != (size_t)n) msg(ERROR, "Failed to read %s.", argv[1]);
	buf[n] = '\0';
	fclose(f);
	dictionary *ini = iniFromString(buf);
	free(buf);
	for (int i = 2; i < argc; i++) {
		char tmp[1024];
		snprintf(tmp, sizeof(tmp), "%s", argv[i]);
		char *eq = strchr(tmp, '=');
		if (!eq) msg(ERROR, "override without '=': %s", argv[i]);
		*eq = '\0';
		iniSet(ini, tmp, eq + 1);
	}
	return ini;
}

void iniClose(dictionary *ini) {
	if (!ini) return;
	for (int i = 0; i < ini->n; i++) {
		free(ini->e[i].key);
		free(ini->e[i].val);
	}
	free(ini->e);
	free(ini);
}

static const char *lookup(const dictionary *ini, const char *key) {
	char k[512];
	snprintf(k, sizeof(k), "%s", key);
	lowercase(k);
	for (int i = 0; i < ini->n; i++)
		if (!strcmp(ini->e[i].key, k)) return ini->e[i].val;
	return NULL;
}

int iniHas(const dictionary *ini, const char *key) { return lookup(ini, key) != NULL; }

static const char *req(const dictionary *ini, const char *key) {
	const char *v = lookup(ini, key);
	if (!v) msg(ERROR, "Key \"%s\" not found in input file", key);
	return v;
}

int iniGetNElements(const dictionary *ini, const char *key) {
	const char *v = req(ini, key);
	if (!v[0]) return 0;
	int n = 1;
	for (; *v; v++) n += (*v == ',');
	return n;
}

int iniGetInt(const dictionary *ini, const char *key) { return (int)atof(req(ini, key)); }
long iniGetLongInt(const dictionary *ini, const char *key) { return (long)atof(req(ini, key)); }
double iniGetDouble(const dictionary *ini, const char *key) { return atof(req(ini, key)); }
char *iniGetStr(const dictionary *ini, const char *key) { return dupstr(req(ini, key)); }

void freeStrArr(char **a) {
	for (int i = 0; a[i]; i++) free(a[i]);
	free(a);
}

static char **splitList(const char *list, int *count) {
	int cap = 2;
	for (const char *t = list; *t; t++) cap += (*t == ',');
	char **r = malloc(cap * sizeof(char *));
	int n = 0;
	const char *start = list;
	for (const char *t = list;; t++) {
		if (*t == ',' || *t == '\0') {
			const char *a = start, *b = t - 1;
			while (*a == ' ' && a < b) a++;
			while (*b == ' ' && a < b) b--;
			int len = (int)(b - a + 1);
			if (len < 0) len = 0;
			r[n] = malloc(len + 1);
			memcpy(r[n], a, len);
			r[n][len] = '\0';
			n++;
			start = t + 1;
			if (!*t) break;
		}
	}
	r[n] = NULL;
	*count = n;
	return r;
}

char **iniGetStrArr(const dictionary *ini, const char *key, int nElements) {
	int m;
	char **base = splitList(req(ini, key), &m);
	char **r = malloc((nElements + 1) * sizeof(char *));
	for (int i = 0; i < nElements; i++) r[i] = dupstr(base[i % m]);
	r[nElements] = NULL;
	freeStrArr(base);
	return r;
}

int *iniGetIntArr(const dictionary *ini, const char *key, int n) {
	char **s = iniGetStrArr(ini, key, n);
	int *r = malloc(n * sizeof(int));
	for (int i = 0; i < n; i++) r[i] = (int)atof(s[i]);
	freeStrArr(s);
	return r;
}

long *iniGetLongIntArr(const dictionary *ini, const char *key, int n) {
	char **s = iniGetStrArr(ini, key, n);
	long *r = malloc(n * sizeof(long));
	for (int i = 0; i < n; i++) r[i] = (long)atof(s[i]);
	freeStrArr(s);
	return r;
}

double *iniGetDoubleArr(const dictionary *ini, const char *key, int n) {
	char **s = iniGetStrArr(ini, key, n);
	double *r = malloc(n * sizeof(double));
	for (int i = 0; i < n; i++) r[i] = atof(s[i]);
	freeStrArr(s);
	return r;
}

void iniSetDoubleArr(dictionary *ini, const char *key, const double *v, int n) {
	char list[4096] = "", num[64];
	for (int i = 0; i < n; i++) {
		snprintf(num, sizeof(num), i ? ",%a" : "%a", v[i]);
		strcat(list, num);
	}
	iniSet(ini, key, list);
}

void iniSetDouble(dictionary *ini, const char *key, double v) {
	char num[64];
	snprintf(num, sizeof(num), "%a", v);
	iniSet(ini, key, num);
}

void iniScaleDouble(dictionary *ini, const char *key, double factor) {
	int n = iniGetNElements(ini, key);
	double *a = iniGetDoubleArr(ini, key, n);
	for (int i = 0; i < n; i++) a[i] *= factor;
	iniSetDoubleArr(ini, key, a, n);
	free(a);
}

void iniApplySuffix(dictionary *ini, const char *key, const char *suffix, const double *mul, int mulLen) {
	int n = iniGetNElements(ini, key);
	char **s = iniGetStrArr(ini, key, n);
	double *a = malloc(n * sizeof(double));
	for (int i = 0; i < n; i++) {
		a[i] = atof(s[i]);
		if (strstr(s[i], suffix)) a[i] *= mul[i % mulLen];
	}
	iniSetDoubleArr(ini, key, a, n);
	free(a);
	freeStrArr(s);
}

/* io.c:115-168: match the ini value against the stringified "name_set" list */
funPtr selectInner(const dictionary *ini, const char *key, const char *list, ...) {
	va_list args;
	va_start(args, list);
	const char *value = req(ini, key);
	int n;
	char **names = splitList(list, &n);
	funPtr (*chosen)() = NULL;
	for (int i = 0; i < n; i++) {
		char *nm = trim(names[i]);
		char *us = strstr(nm, "_set");
		if (us) *us = '\0';
		funPtr (*fun)() = va_arg(args, funPtr (*)());
		if (!strcmp(nm, value)) chosen = fun;
	}
	va_end(args);
	if (!chosen) {
		char valid[1024] = "";
		for (int i = 0; i < n; i++) {
			strcat(valid, " ");
			strcat(valid, trim(names[i]));
		}
		freeStrArr(names);
		msg(ERROR, "%s=%s invalid. Valid arguments:%s.", key, value, valid);
	}
	freeStrArr(names);
	return chosen((dictionary *)ini);
}

/* -------------------------------------------------------------- units -- */
static const double elementaryCharge = 1.60217733e-19;
static const double electronMass = 9.10938188e-31;
static const double vacuumPermittivity = 8.854187817e-12;

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

static Units *unitsSI(const dictionary *ini) {
	int nd = iniGetInt(ini, "grid:nDims");
	int ns = iniGetInt(ini, "population:nSpecies");
	double timeStep = iniGetDouble(ini, "time:timeStep");
	double *stepSize = iniGetDoubleArr(ini, "grid:stepSize", nd);
	long *nPart = iniGetLongIntArr(ini, "population:nParticles", ns);
	double *density = iniGetDoubleArr(ini, "population:density", ns);
	double *charge = iniGetDoubleArr(ini, "population:charge", ns);
	int L[3];
	long Vl;
	globalSize(ini, nd, L, &Vl);
	double V = Vl * pow(stepSize[0], nd);
	Units *u = calloc(1, sizeof(*u));
	u->weights = malloc(ns * sizeof(double));
	for (int s = 0; s < ns; s++) u->weights[s] = density[s] * V / nPart[s];
	u->nDims = nd;
	u->nSpecies = ns;
	u->length = stepSize[0];
	u->time = timeStep;
	u->charge = u->weights[0] * fabs(charge[0]);
	u->mass = pow(u->time * u->charge, 2) / (vacuumPermittivity * pow(u->length, nd));
	free(stepSize);
	free(nPart);
	free(density);
	free(charge);
	return u;
}

Units *uAlloc(dictionary *ini) {
	/* parseIndirectInput (units.c:138-157) */
	int nd = iniGetInt(ini, "grid:nDims");
	int L[3];
	long Vl;
	globalSize(ini, nd, L, &Vl);
	double V = (double)Vl, mul[3];
	for (int i = 0; i < nd; i++) mul[i] = 1.0 / L[i];
	iniApplySuffix(ini, "population:nParticles", "pc", &V, 1);
	iniApplySuffix(ini, "population:nAlloc", "pc", &V, 1);
	iniApplySuffix(ini, "grid:nEmigrantsAlloc", "pc", &V, 1);
	iniApplySuffix(ini, "grid:stepSize", "tot", mul, nd);
	const char *method = req(ini, "methods:normalization");
	Units *u = NULL;
	if (!strcmp(method, "semiSI")) {
		int ns = iniGetInt(ini, "population:nSpecies");
		double *charge = iniGetDoubleArr(ini, "population:charge", ns);
		double *mass = iniGetDoubleArr(ini, "population:mass", ns);
		double *density = iniGetDoubleArr(ini, "population:density", ns);
		double timeStep = iniGetDouble(ini, "time:timeStep");
		if (fabs(charge[0] + 1) > 1e-10) msg(ERROR, "Species 0 must have charge -1 with this normalization");
		if (fabs(mass[0] - 1) > 1e-10) msg(ERROR, "Species 0 must have mass 1 with this normalization");
		for (int s = 0; s < ns; s++) {
			charge[s] *= elementaryCharge;
			mass[s] *= electronMass;
		}
		double wpe = sqrt(pow(elementaryCharge, 2) * density[0] / (vacuumPermittivity * electronMass));
		timeStep /= wpe;
		iniSetDoubleArr(ini, "population:charge", charge, ns);
		iniSetDoubleArr(ini, "population:mass", mass, ns);
		iniSetDouble(ini, "time:timeStep", timeStep);
		free(charge);
		free(mass);
		free(density);
		u = unitsSI(ini);
	} else if (!strcmp(method, "SI")) {
		u = unitsSI(ini);
	} else {
		msg(ERROR, "methods:normalization not valid (must be SI or semiSI)");
	}
	double X = u->length, T = u->time, Q = u->charge, M = u->mass, D = u->nDims;
	u->hyperArea = pow(X, D - 1);
	u->hyperVolume = pow(X, D);
	u->frequency = 1.0 / T;
	u->velocity = X / T;
	u->acceleration = X / pow(T, 2);
	u->density = 1.0 / pow(X, D);
	u->chargeDensity = Q / pow(X, D);
	u->potential = pow(X / T, 2) * M / Q;
	u->eField = X * M / (pow(T, 2) * Q);
	u->bField = M / (T * Q);
	u->energy = M * pow(X / T, 2);
	return u;
}

void uFree(Units *u) {
	if (!u) return;
	free(u->weights);
	free(u);
}

void uNormalize(dictionary *ini, const Units *u) {
	int ns = u->nSpecies;
	double *c = iniGetDoubleArr(ini, "population:charge", ns);
	double *m = iniGetDoubleArr(ini, "population:mass", ns);
	double *dn = iniGetDoubleArr(ini, "population:density", ns);
	for (int s = 0; s < ns; s++) {
		c[s] *= u->weights[s];
		m[s] *= u->weights[s];
		dn[s] /= u->weights[s];
	}
	for (int s = 0; s < ns; s++) {
		c[s] *= 1.0 / u->charge;
		m[s] *= 1.0 / u->mass;
		dn[s] *= 1.0 / u->density;
	}
	iniSetDoubleArr(ini, "population:charge", c, ns);
	iniSetDoubleArr(ini, "population:mass", m, ns);
	iniSetDoubleArr(ini, "population:density", dn, ns);
	free(c);
	free(m);
	free(dn);
	iniScaleDouble(ini, "population:thermalVelocity", 1.0 / u->velocity);
	iniScaleDouble(ini, "population:drift", 1.0 / u->velocity);
	iniScaleDouble(ini, "population:perturbAmplitude", 1.0 / u->length);
	iniScaleDouble(ini, "fields:BExt", 1.0 / u->bField);
	iniScaleDouble(ini, "fields:EExt", 1.0 / u->eField);
}

/* ------------------------------------------------------------ context -- */
/* the device context of this process; its world (rank, size, device) comes
 * from the PincSim options or, for a main.c-style caller, from the launcher
 * (pinc_boot.c) */
void pinc_ctx_init(void) {
	if (g_pinc.initialised) return;
	pinc_check(pinc_hip_set_device(g_pinc.device), "set device");
	pinc_check(pinc_hip_stream_create(&g_pinc.stream), "stream");
	pinc_check(pinc_hip_malloc((void **)&g_pinc.dScratch, (PINC_PARTIALS + 256) * sizeof(double)),
	           "scratch");
	pinc_check(pinc_hip_malloc((void **)&g_pinc.dErr, 64), "err word");
	pinc_check(pinc_hip_host_alloc((void **)&g_pinc.hPinned, 32 * sizeof(double)), "pinned host scratch");
	pinc_check(pinc_hip_memset(g_pinc.dErr, 0, 64, g_pinc.stream), "err word");
	if (g_pinc.nranks < 1) g_pinc.nranks = 1;
	g_pinc.verbose = getenv("PINC_VERBOSE") ? atoi(getenv("PINC_VERBOSE")) : 0;
	g_pinc.traceSort = getenv("PINC_TRACE_SORT") ? atoi(getenv("PINC_TRACE_SORT")) : 0;
	g_pinc.extractSkip = !(getenv("PINC_EXTRACT_SKIP") && !atoi(getenv("PINC_EXTRACT_SKIP")));
	g_pinc.flagsSparse = !(getenv("PINC_FLAGS_SPARSE") && !atoi(getenv("PINC_FLAGS_SPARSE")));
	for (int p = 0; p < PINC_NPHASES; p++)
		for (int i = 0; i < 2 * PINC_PHASE_RING; i++) pinc_check(pinc_hip_event_create(&g_pinc.ev[p][i]), "event");
	g_pinc.initialised = 1;
}

void pinc_ctx_require(void) {
	if (g_pinc.initialised) return;
	pinc_boot_world();
}

/* phase timers (PincSimOpts.timing): an event pair per phase interval,
 * summed into phaseMs only when the ring of a phase is full or the totals
 * are read, so that timing adds no host wait to the step (an elapsed time
 * waits for its stop event) */
void pinc_phase_begin(int p) {
	if (!g_pinc.timing) return;
	pinc_check(pinc_hip_event_record(g_pinc.ev[p][2 * g_pinc.phaseN[p]], g_pinc.stream), "event");
	g_pinc.phaseOpen[p] = 1;
}

static void phase_flush(int p) {
	for (int i = 0; i < g_pinc.phaseN[p]; i++) {
		float ms = 0;
		pinc_check(pinc_hip_event_elapsed(&ms, g_pinc.ev[p][2 * i], g_pinc.ev[p][2 * i + 1]), "elapsed");
		g_pinc.phaseMs[p] += ms;
	}
	g_pinc.phaseN[p] = 0;
}

void pinc_phase_end(int p) {
	if (!g_pinc.timing || !g_pinc.phaseOpen[p]) return;
	pinc_check(pinc_hip_event_record(g_pinc.ev[p][2 * g_pinc.phaseN[p] + 1], g_pinc.stream), "event");
	g_pinc.phaseOpen[p] = 0;
	if (++g_pinc.phaseN[p] == PINC_PHASE_RING) phase_flush(p);
}

void pinc_phase_flush(void) {
	if (!g_pinc.initialised) return;
	for (int p = 0; p < PINC_NPHASES; p++)
		if (!g_pinc.phaseOpen[p]) phase_flush(p);
}

/* ------------------------------------------------------------- probe -- */
static void probe_release(void) {
	for (int k = 0; k < PINC_NPROBES; k++) {
		if (g_pinc.probeEv[k]) {
			for (int i = 0; i < 2 * g_pinc.probeMax; i++) pinc_hip_event_destroy(g_pinc.probeEv[k][i]);
			free(g_pinc.probeEv[k]);
			free(g_pinc.probeBytes[k]);
			free(g_pinc.probeTag[k]);
		}
		g_pinc.probeEv[k] = NULL;
		g_pinc.probeBytes[k] = NULL;
		g_pinc.probeTag[k] = NULL;
		g_pinc.probeOn[k] = 0;
		g_pinc.probeN[k] = 0;
		g_pinc.probeLaunches[k] = 0;
	}
}

int pinc_probe_start(int kernel, int maxSamples) {
	pinc_ctx_require();
	if (kernel < PINC_PROBE_ALL || kernel >= PINC_NPROBES || maxSamples < 1) return 1;
	probe_release();
	g_pinc.probeMax = maxSamples;
	for (int k = 0; k < PINC_NPROBES; k++) {
		if (kernel != PINC_PROBE_ALL && kernel != k) continue;
		g_pinc.probeOn[k] = 1;
		g_pinc.probeEv[k] = calloc(2 * maxSamples, sizeof(void *));
		g_pinc.probeBytes[k] = calloc(maxSamples, sizeof(double));
		g_pinc.probeTag[k] = calloc(maxSamples, sizeof(int));
		for (int i = 0; i < 2 * maxSamples; i++)
			pinc_check(pinc_hip_event_create(&g_pinc.probeEv[k][i]), "probe event");
	}
	return 0;
}

/* a launch of probe k that is not timed (sampling every launch would put an
 * event record, ~5 us of host time, between back-to-back kernels): counted
 * so that launches x mean time is the kernel's whole cost */
void pinc_probe_count(int k) {
	if (g_pinc.probeOn[k] && !g_pinc.capturing) g_pinc.probeLaunches[k]++;
}

int pinc_probe_begin(int k) {
	if (!g_pinc.probeOn[k] || g_pinc.capturing) return -1;
	g_pinc.probeLaunches[k]++;
	if (g_pinc.probeN[k] >= g_pinc.probeMax) return -1;
	int slot = g_pinc.probeN[k]++;
	pinc_check(pinc_hip_event_record(g_pinc.probeEv[k][2 * slot], g_pinc.stream), "probe");
	return slot;
}

void pinc_probe_end(int k, int slot, double bytes) {
	if (slot < 0 || !g_pinc.probeOn[k]) return;
	pinc_check(pinc_hip_event_record(g_pinc.probeEv[k][2 * slot + 1], g_pinc.stream), "probe");
	g_pinc.probeBytes[k][slot] = bytes;
}

void pinc_probe_tag(int k, int slot, int tag) {
	if (slot >= 0 && g_pinc.probeOn[k]) g_pinc.probeTag[k][slot] = tag;
}

int pinc_probe_sample(int k, int i, double *ms, int *tag) {
	if (k < 0 || k >= PINC_NPROBES || !g_pinc.probeOn[k] || i < 0 || i >= g_pinc.probeN[k]) return 1;
	float t = 0;
	pinc_check(pinc_hip_event_elapsed(&t, g_pinc.probeEv[k][2 * i], g_pinc.probeEv[k][2 * i + 1]), "probe read");
	*ms = t;
	*tag = g_pinc.probeTag[k][i];
	return 0;
}

int pinc_probe_read(int k, double *meanMs, double *meanBytes, int *samples, long *launches) {
	if (k < 0 || k >= PINC_NPROBES) return 1;
	double t = 0, b = 0;
	int n = g_pinc.probeOn[k] ? g_pinc.probeN[k] : 0;
	for (int i = 0; i < n; i++) {
		float ms = 0;
		pinc_check(pinc_hip_event_elapsed(&ms, g_pinc.probeEv[k][2 * i], g_pinc.probeEv[k][2 * i + 1]),
		           "probe read");
		t += ms;
		b += g_pinc.probeBytes[k][i];
	}
	*meanMs = n ? t / n : 0;
	*meanBytes = n ? b / n : 0;
	*samples = n;
	*launches = g_pinc.probeLaunches[k];
	return 0;
}

/* reduce the first nParts partials in the scratch area into slot 0; read it */
double pinc_reduce_host(int nParts, double div) {
	pinc_check(pinc_hip_reduce(g_pinc.dScratch, nParts, div, PINC_SLOT(0), g_pinc.stream), "reduce");
	double v = 0;
	pinc_check(pinc_hip_d2h(&v, PINC_SLOT(0), sizeof(double), g_pinc.stream), "reduce readback");
	return v;
}

/* -------------------------------------------------------------- timer -- */
/* aux.c:48-85 (Timer, core.h:419-436).  The operators queue device work, so
 * tStop first waits for the stream: a tStart/tStop span then covers the work
 * issued inside it, as the reference's blocking loop did. */
#include <time.h>
static long long now_ns(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (long long)t.tv_sec * 1000000000LL + t.tv_nsec;
}

Timer *tAlloc() {
	Timer *t = malloc(sizeof(*t));
	t->start = 0;
	t->total = 0;
	return t;
}

void tFree(Timer *t) { free(t); }

void tStart(Timer *t) {
	if (g_pinc.initialised) pinc_check(pinc_hip_stream_sync(g_pinc.stream), "tStart");
	t->start = now_ns();
}

void tStop(Timer *t) {
	if (g_pinc.initialised) pinc_check(pinc_hip_stream_sync(g_pinc.stream), "tStop");
	t->total += now_ns() - t->start;
}

void tReset(Timer *t) { t->total = 0; }

void tMsg(long long nanoSec, const char *string) {
	if (nanoSec >= 1000000000LL) msg(TIMER, "%s %6.2fs ", string, (double)nanoSec / 1e9);
	else if (nanoSec > 1000000LL) msg(TIMER, "%s %6.2fms ", string, (double)nanoSec / 1e6);
	else if (nanoSec > 1000LL) msg(TIMER, "%s %6.2fus ", string, (double)nanoSec / 1e3);
	else msg(TIMER, "%s %6.2fns ", string, (double)nanoSec);
}
