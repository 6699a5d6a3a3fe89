/*
 * pinc_comm.c -- the three collectives the hot path needs, over RCCL or over
 * a host transport.
 *
 *   exchange        paired point-to-point sends/receives (z-slab halo planes,
 *                   migrant counts and records; pusher.c:914-1027 and
 *                   grid.c:392-402 for the reference's MPI_Sendrecv use)
 *   allgather       rho slabs -> global rho for the replicated solve
 *   allreduce_sum   neutralisation sums and energies (MPI_Allreduce)
 *
 * Default: RCCL over xGMI on the library's stream (device buffers, no host
 * round trip).  pinc_set_host_transport() installs callbacks that move host
 * buffers instead; the device data is staged through pinned host memory.
 * That path exists so the multi-rank code runs with several processes on
 * one GPU (RCCL refuses duplicate devices) and in CI; it is never the
 * default and never used by the bench.
 */
#include "pinc_internal.h"

/* PINC_COMM_TRACE=<dir>: every collective this rank issues, in issue order,
 * one line each in <dir>/comm_rank<r>.log (kind, sequence number, caller's
 * label, peers and byte counts), flushed per line, whichever transport
 * carries it.  RCCL pairs point-to-point calls per peer in issue order and
 * needs every rank to issue the same collectives in the same order; gloo
 * matches by tag and is more forgiving, so the host-transport rehearsal
 * records the sequence and tools/comm_pairing.py checks it under RCCL's
 * rules (tests/test_gpu_comm_pairing.py). */
static FILE *g_trace = NULL;
static int g_traceInit = 0;
static long g_traceSeq = 0;

static FILE *trace_file(void) {
	if (!g_traceInit) {
		g_traceInit = 1;
		const char *d = getenv("PINC_COMM_TRACE");
		if (d && *d) {
			char path[4096];
			snprintf(path, sizeof(path), "%s/comm_rank%d.log", d, g_pinc.rank);
			g_trace = fopen(path, "w");
			if (!g_trace) msg(ERROR, "PINC_COMM_TRACE: cannot write %s", path);
		}
	}
	return g_trace;
}

/* Per-kind statistics of the collectives (pinc_comm_stats_start/read; the
 * bench's multi-rank line): calls, this rank's payload bytes (exchange: the
 * bytes it sends; allgather: its own contribution; allreduce: the vector),
 * and device time between HIP events recorded around each call on the
 * library's stream (RCCL runs there; the host transport's staging copies
 * too), read lazily so nothing synchronises inside the timed region. */
static const char *const g_kindName[PINC_COMM_KINDS] = {"halo", "ext_halo", "migrate", "allgather", "allreduce",
                                                         "spectral_transpose"};
static int g_statOn = 0, g_statCap = 0, g_statN = 0;
static void **g_statEv = NULL;
static int *g_statKind = NULL;
static double g_statBytes[PINC_COMM_KINDS];
static long g_statCalls[PINC_COMM_KINDS];

static int exchange_kind(const char *what) {
	if (strstr(what, "ext halo")) return 1;
	if (strstr(what, "halo")) return 0;
	if (strstr(what, "count") || strstr(what, "migrant")) return 2;
	return 5; /* the slab-distributed spectral solve's all-to-all */
}

int pinc_comm_stats_start(int maxCalls) {
	pinc_ctx_require();
	if (maxCalls < 1) maxCalls = 1;
	if (maxCalls > g_statCap) {
		void **ev = realloc(g_statEv, 2 * (size_t)maxCalls * sizeof(void *));
		int *kd = realloc(g_statKind, (size_t)maxCalls * sizeof(int));
		if (!ev || !kd) msg(ERROR, "comm stats: out of memory");
		g_statEv = ev;
		g_statKind = kd;
		for (int i = 2 * g_statCap; i < 2 * maxCalls; i++) pinc_check(pinc_hip_event_create(&g_statEv[i]), "comm stats");
		g_statCap = maxCalls;
	}
	g_statN = 0;
	for (int k = 0; k < PINC_COMM_KINDS; k++) {
		g_statBytes[k] = 0;
		g_statCalls[k] = 0;
	}
	g_statOn = 1;
	return 0;
}

static int stat_begin(int kind, double bytes) {
	if (!g_statOn) return -1;
	g_statCalls[kind]++;
	g_statBytes[kind] += bytes;
	if (g_statN >= g_statCap || g_pinc.capturing) return -1;
	int slot = g_statN++;
	g_statKind[slot] = kind;
	pinc_check(pinc_hip_event_record(g_statEv[2 * slot], g_pinc.stream), "comm stats");
	return slot;
}

static void stat_end(int slot) {
	if (slot >= 0) pinc_check(pinc_hip_event_record(g_statEv[2 * slot + 1], g_pinc.stream), "comm stats");
}

/* per kind: device ms (timed calls), payload bytes and calls since the start;
 * returns the number of kinds, or -1 if statistics were never started */
int pinc_comm_stats_read(double *ms, double *bytes, long *calls, long *timedCalls) {
	if (!g_statCap) return -1;
	for (int k = 0; k < PINC_COMM_KINDS; k++) {
		ms[k] = 0;
		bytes[k] = g_statBytes[k];
		calls[k] = g_statCalls[k];
		if (timedCalls) timedCalls[k] = 0;
	}
	for (int i = 0; i < g_statN; i++) {
		float t = 0;
		pinc_check(pinc_hip_event_elapsed(&t, g_statEv[2 * i], g_statEv[2 * i + 1]), "comm stats read");
		ms[g_statKind[i]] += t;
		if (timedCalls) timedCalls[g_statKind[i]]++;
	}
	return PINC_COMM_KINDS;
}

const char *pinc_comm_kind_name(int kind) { return kind >= 0 && kind < PINC_COMM_KINDS ? g_kindName[kind] : ""; }

static pinc_host_transport_t g_tr;
static int g_trSet = 0;
static unsigned char *g_stage = NULL;
static long g_stageCap = 0;

int pinc_set_host_transport(const pinc_host_transport_t *t) {
	if (t) {
		g_tr = *t;
		g_trSet = 1;
	} else {
		memset(&g_tr, 0, sizeof(g_tr));
		g_trSet = 0;
	}
	return 0;
}

int pinc_comm_host_transport(void) { return g_trSet; }

static unsigned char *stage(long bytes) {
	if (bytes > g_stageCap) {
		free(g_stage);
		g_stageCap = bytes + bytes / 4 + 4096;
		g_stage = malloc(g_stageCap);
		if (!g_stage) msg(ERROR, "host transport: out of memory (%ld bytes)", g_stageCap);
	}
	return g_stage;
}

void pinc_comm_exchange(int nOps, const int *sendPeer, void *const *sendbuf, const long *sendBytes,
                        const int *recvPeer, void *const *recvbuf, const long *recvBytes, const char *what) {
	FILE *tf = trace_file();
	if (tf) {
		fprintf(tf, "X %ld %s|%d", g_traceSeq++, what, nOps);
		for (int i = 0; i < nOps; i++) fprintf(tf, " s%d:%ld r%d:%ld", sendPeer[i], sendBytes[i], recvPeer[i], recvBytes[i]);
		fputc('\n', tf);
		fflush(tf);
	}
	double sent = 0;
	for (int i = 0; i < nOps; i++) sent += (double)sendBytes[i];
	const int slot = stat_begin(exchange_kind(what), sent);
	if (!g_trSet) {
		pinc_hip_comm_note(what);
		pinc_check(pinc_hip_comm_exchange(g_pinc.comm, nOps, sendPeer, sendbuf, sendBytes, recvPeer, recvbuf,
		                                  recvBytes, g_pinc.stream),
		           what);
		stat_end(slot);
		return;
	}
	long tot = 0;
	for (int i = 0; i < nOps; i++) tot += sendBytes[i] + recvBytes[i];
	unsigned char *h = stage(tot);
	const void **hs = malloc(nOps * sizeof(*hs));
	void **hr = malloc(nOps * sizeof(*hr));
	if (!hs || !hr) msg(ERROR, "host transport: out of memory");
	long off = 0;
	for (int i = 0; i < nOps; i++) {
		hs[i] = h + off;
		if (sendBytes[i]) pinc_check(pinc_hip_d2h(h + off, sendbuf[i], sendBytes[i], g_pinc.stream), what);
		off += sendBytes[i];
	}
	for (int i = 0; i < nOps; i++) {
		hr[i] = h + off;
		off += recvBytes[i];
	}
	if (g_tr.exchange(g_tr.user, nOps, sendPeer, hs, sendBytes, recvPeer, hr, recvBytes))
		msg(ERROR, "host transport exchange failed (%s)", what);
	for (int i = 0; i < nOps; i++)
		if (recvBytes[i]) pinc_check(pinc_hip_h2d(recvbuf[i], hr[i], recvBytes[i], g_pinc.stream), what);
	free(hs);
	free(hr);
	stat_end(slot);
}

void pinc_comm_allgather(const double *send, double *recv, long count, const char *what) {
	FILE *tf = trace_file();
	if (tf) {
		fprintf(tf, "G %ld %s|%ld\n", g_traceSeq++, what, count);
		fflush(tf);
	}
	const int slot = stat_begin(3, (double)count * sizeof(double));
	if (!g_trSet) {
		pinc_hip_comm_note(what);
		pinc_check(pinc_hip_comm_allgather(g_pinc.comm, send, recv, count, g_pinc.stream), what);
		stat_end(slot);
		return;
	}
	long sb = count * (long)sizeof(double);
	unsigned char *h = stage(sb * (g_pinc.nranks + 1));
	pinc_check(pinc_hip_d2h(h, send, sb, g_pinc.stream), what);
	if (g_tr.allgather(g_tr.user, (const double *)h, (double *)(h + sb), count))
		msg(ERROR, "host transport allgather failed (%s)", what);
	pinc_check(pinc_hip_h2d(recv, h + sb, sb * g_pinc.nranks, g_pinc.stream), what);
	stat_end(slot);
}

void pinc_comm_allreduce_sum(double *buf, long count, const char *what) {
	FILE *tf = trace_file();
	if (tf) {
		fprintf(tf, "R %ld %s|%ld\n", g_traceSeq++, what, count);
		fflush(tf);
	}
	const int slot = stat_begin(4, (double)count * sizeof(double));
	if (!g_trSet) {
		pinc_hip_comm_note(what);
		pinc_check(pinc_hip_comm_allreduce_sum(g_pinc.comm, buf, buf, count, g_pinc.stream), what);
		stat_end(slot);
		return;
	}
	long sb = count * (long)sizeof(double);
	double *h = (double *)stage(sb);
	pinc_check(pinc_hip_d2h(h, buf, sb, g_pinc.stream), what);
	if (g_tr.allreduce_sum(g_tr.user, h, count)) msg(ERROR, "host transport allreduce failed (%s)", what);
	pinc_check(pinc_hip_h2d(buf, h, sb, g_pinc.stream), what);
	stat_end(slot);
}
