/*
 * pinc_boot.c -- the process world of the reference's main.c without MPI in
 * this library: rank, size and device from the launcher, and the transport
 * for the three collectives of pinc_comm.c.
 *
 * The reference calls MPI_Init in main() (main.c:24) and reads the world in
 * gAllocMpi (grid.c:502-545: MPI_Comm_rank / MPI_Comm_size).  This library
 * needs no MPI: gAllocMpi (and regular()) call pinc_boot_world(), which
 *
 *   1. reads rank / size / local rank from the launcher's environment, first
 *      match wins: PINC_RANK / PINC_WORLD_SIZE / PINC_LOCAL_RANK; torchrun
 *      (RANK, WORLD_SIZE, LOCAL_RANK); Open MPI (OMPI_COMM_WORLD_*); MPICH /
 *      Intel MPI hydra (PMI_RANK, PMI_SIZE, MPI_LOCALRANKID); Slurm
 *      (SLURM_PROCID, SLURM_NTASKS, SLURM_LOCALID).  None set: one rank.
 *   2. selects the GPU: PINC_DEVICE, else local rank mod the visible devices
 *      (one process per GPU, as PINC runs one MPI rank per core).
 *   3. with several ranks, meets the others over TCP on PINC_MASTER_ADDR
 *      (else MASTER_ADDR, else 127.0.0.1) port PINC_MASTER_PORT (else
 *      MASTER_PORT + 1 -- torchrun's own store holds MASTER_PORT -- else
 *      29533).  Rank 0 listens, every other rank connects within
 *      PINC_BOOT_TIMEOUT seconds (default 120).  Then either
 *        - RCCL (default): rank 0 makes the 128-byte ncclUniqueId and sends it
 *          over these sockets, every rank joins the communicator; or
 *        - PINC_TRANSPORT=host: the ranks open a full TCP mesh and the
 *          collectives run over it through pinc_set_host_transport (device
 *          data staged through host memory).  This is the path for several
 *          ranks on one GPU (RCCL refuses duplicate devices), e.g. the
 *          two-rank C driver test, and for CI.  Never the bench's transport.
 *
 * A process driven through the PincSim API (pinc_sim_create with explicit
 * PincSimOpts) keeps what its caller configured; nothing is read here.
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

static int g_booted = 0;
static int g_configured = 0;  /* PincSim opts set the world explicitly */
static int *g_peer = NULL;    /* socket to each rank (host transport), -1 for self */
static int g_nPeer = 0;

void pinc_boot_configured(void) { g_configured = 1; }
/* exported: the caller sets the world through PincSimOpts (Python, bench) */
void pinc_world_explicit(void) { g_configured = 1; }

static const char *env_first(const char *const *names) {
	for (int i = 0; names[i]; i++) {
		const char *v = getenv(names[i]);
		if (v && *v) return v;
	}
	return NULL;
}

/* launcher families, each a (rank, size, local rank) triple of variables */
static const char *const g_env[][3] = {
	{"PINC_RANK", "PINC_WORLD_SIZE", "PINC_LOCAL_RANK"},
	{"RANK", "WORLD_SIZE", "LOCAL_RANK"},
	{"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"},
	{"PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"},
	{"SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"},
};

/* rank, size and local rank of this process from the launcher (size 1 if
 * none is found); returns the family's rank variable or NULL */
const char *pinc_launcher_env(int *rank, int *size, int *local) {
	*rank = 0;
	*size = 1;
	*local = 0;
	for (size_t f = 0; f < sizeof(g_env) / sizeof(g_env[0]); f++) {
		const char *r = getenv(g_env[f][0]), *s = getenv(g_env[f][1]);
		if (!r || !*r || !s || !*s) continue;
		*rank = atoi(r);
		*size = atoi(s);
		const char *l = getenv(g_env[f][2]);
		*local = l && *l ? atoi(l) : *rank;
		if (*size < 1 || *rank < 0 || *rank >= *size)
			msg(ERROR | ALL, "launcher environment %s=%s %s=%s is not a valid world", g_env[f][0], r, g_env[f][1], s);
		return g_env[f][0];
	}
	return NULL;
}

/* ------------------------------------------------------------- sockets -- */
static double now_s(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void send_all(int fd, const void *buf, size_t n, const char *what) {
	const char *p = buf;
	while (n) {
		ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
		if (k < 0 && (errno == EINTR || errno == EAGAIN)) {
			struct pollfd q = {fd, POLLOUT, 0};
			poll(&q, 1, 1000);
			continue;
		}
		if (k <= 0) msg(ERROR | ALL, "[pinc rank %d] %s: send failed (%s)", g_pinc.rank, what, strerror(errno));
		p += k;
		n -= (size_t)k;
	}
}

static void recv_all(int fd, void *buf, size_t n, const char *what) {
	char *p = buf;
	while (n) {
		ssize_t k = recv(fd, p, n, 0);
		if (k < 0 && (errno == EINTR || errno == EAGAIN)) {
			struct pollfd q = {fd, POLLIN, 0};
			poll(&q, 1, 1000);
			continue;
		}
		if (k == 0) msg(ERROR | ALL, "[pinc rank %d] %s: peer closed the connection", g_pinc.rank, what);
		if (k < 0) msg(ERROR | ALL, "[pinc rank %d] %s: recv failed (%s)", g_pinc.rank, what, strerror(errno));
		p += k;
		n -= (size_t)k;
	}
}

static void tune(int fd) {
	int one = 1;
	setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

static int listen_on(unsigned short port, unsigned short *bound) {
	int fd = socket(AF_INET, SOCK_STREAM, 0);
	if (fd < 0) msg(ERROR | ALL, "socket: %s", strerror(errno));
	int one = 1;
	setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
	struct sockaddr_in a;
	memset(&a, 0, sizeof(a));
	a.sin_family = AF_INET;
	a.sin_addr.s_addr = htonl(INADDR_ANY);
	a.sin_port = htons(port);
	if (bind(fd, (struct sockaddr *)&a, sizeof(a)))
		msg(ERROR | ALL, "[pinc rank %d] cannot listen on port %u (%s): set PINC_MASTER_PORT", g_pinc.rank, port,
		    strerror(errno));
	if (listen(fd, 64)) msg(ERROR | ALL, "listen: %s", strerror(errno));
	socklen_t len = sizeof(a);
	getsockname(fd, (struct sockaddr *)&a, &len);
	if (bound) *bound = ntohs(a.sin_port);
	return fd;
}

static int accept_by(int lfd, double deadline, const char *what) {
	for (;;) {
		struct pollfd q = {lfd, POLLIN, 0};
		int left = (int)((deadline - now_s()) * 1000);
		if (left <= 0) msg(ERROR | ALL, "[pinc rank %d] %s: timed out waiting for the other ranks", g_pinc.rank, what);
		int r = poll(&q, 1, left < 1000 ? left : 1000);
		if (r <= 0) continue;
		int fd = accept(lfd, NULL, NULL);
		if (fd >= 0) {
			tune(fd);
			return fd;
		}
	}
}

static int connect_by(const char *host, unsigned short port, double deadline, const char *what) {
	char ps[16];
	snprintf(ps, sizeof(ps), "%u", port);
	struct addrinfo hints, *res = NULL;
	memset(&hints, 0, sizeof(hints));
	hints.ai_family = AF_INET;
	hints.ai_socktype = SOCK_STREAM;
	if (getaddrinfo(host, ps, &hints, &res) || !res)
		msg(ERROR | ALL, "[pinc rank %d] %s: cannot resolve %s", g_pinc.rank, what, host);
	for (;;) {
		int fd = socket(AF_INET, SOCK_STREAM, 0);
		if (fd >= 0 && connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
			freeaddrinfo(res);
			tune(fd);
			return fd;
		}
		if (fd >= 0) close(fd);
		if (now_s() > deadline)
			msg(ERROR | ALL, "[pinc rank %d] %s: no rank 0 at %s:%u (%s)", g_pinc.rank, what, host, port,
			    strerror(errno));
		usleep(50000);
	}
}

/* ------------------------------------------------ host transport (TCP) -- */
/* One stream per peer: sends to a peer leave in op order and receives from a
 * peer are read in op order, so op i of the sender pairs with op i of the
 * receiver (pinc_host_transport_t's contract) without tags.  Everything in
 * flight is progressed together with poll, so no ordering of the ops can
 * deadlock. */
typedef struct {
	int peer;
	char *p;
	long left;
	int send;
} Xfer;

static int sock_exchange(void *user, int nOps, const int *sendPeer, const void *const *sendbuf, const long *sendBytes,
                         const int *recvPeer, void *const *recvbuf, const long *recvBytes) {
	(void)user;
	const int me = g_pinc.rank;
	Xfer *x = calloc(2 * (size_t)nOps + 1, sizeof(Xfer));
	int nx = 0;
	/* messages to this rank itself: k-th self send to k-th self receive */
	int sSelf = 0;
	for (int i = 0; i < nOps; i++) {
		if (sendPeer[i] == me) continue;
		if (sendBytes[i] > 0) x[nx++] = (Xfer){sendPeer[i], (char *)sendbuf[i], sendBytes[i], 1};
	}
	for (int i = 0; i < nOps; i++) {
		if (recvPeer[i] == me) {
			int k = -1;
			for (int j = sSelf; j < nOps; j++)
				if (sendPeer[j] == me) {
					k = j;
					break;
				}
			if (k < 0) {
				free(x);
				return 1;
			}
			sSelf = k + 1;
			if (sendBytes[k] != recvBytes[i]) {
				free(x);
				return 1;
			}
			if (recvBytes[i] > 0) memcpy(recvbuf[i], sendbuf[k], recvBytes[i]);
			continue;
		}
		if (recvBytes[i] > 0) x[nx++] = (Xfer){recvPeer[i], (char *)recvbuf[i], recvBytes[i], 0};
	}
	struct pollfd *q = calloc((size_t)g_nPeer * 2 + 1, sizeof(*q));
	/* a peer that stays connected but makes no progress for PINC_COMM_TIMEOUT
	 * seconds (default 300, as the RCCL watchdog; 0 = wait forever) fails the
	 * exchange instead of hanging every rank */
	const double stallMax = getenv("PINC_COMM_TIMEOUT") ? atof(getenv("PINC_COMM_TIMEOUT")) : 300.0;
	struct timespec t0;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		/* the first unfinished send and receive of each peer */
		int nq = 0, busy = 0;
		for (int r = 0; r < g_nPeer; r++) {
			if (r == me) continue;
			short ev = 0;
			for (int k = 0; k < nx; k++)
				if (x[k].peer == r && x[k].left > 0) ev |= x[k].send ? POLLOUT : POLLIN;
			if (!ev) continue;
			busy = 1;
			q[nq].fd = g_peer[r];
			q[nq].events = ev;
			q[nq].revents = 0;
			nq++;
		}
		if (!busy) break;
		int ready = poll(q, nq, 1000);
		if (ready < 0 && errno != EINTR) {
			free(q);
			free(x);
			return 1;
		}
		struct timespec t1;
		clock_gettime(CLOCK_MONOTONIC, &t1);
		if (ready > 0) t0 = t1;
		else if (stallMax > 0 && (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec) > stallMax) {
			fprintf(stderr, "[pinc] rank %d: host transport exchange made no progress for %.0f s (PINC_COMM_TIMEOUT)\n",
			        me, stallMax);
			free(q);
			free(x);
			return 1;
		}
		for (int j = 0; j < nq; j++) {
			/* a hang-up with sends still pending can never complete them */
			if ((q[j].revents & (POLLERR | POLLNVAL)) ||
			    ((q[j].revents & POLLHUP) && (q[j].events & POLLOUT) && !(q[j].revents & POLLOUT))) {
				free(q);
				free(x);
				return 1;
			}
			int r = -1;
			for (int t = 0; t < g_nPeer; t++)
				if (g_peer[t] == q[j].fd) r = t;
			for (int dir = 1; dir >= 0; dir--) {
				if (dir && !(q[j].revents & POLLOUT)) continue;
				if (!dir && !(q[j].revents & (POLLIN | POLLHUP))) continue;
				for (int k = 0; k < nx; k++) {
					if (x[k].peer != r || x[k].send != dir || x[k].left <= 0) continue;
					ssize_t n = dir ? send(q[j].fd, x[k].p, (size_t)x[k].left, MSG_NOSIGNAL | MSG_DONTWAIT)
					                : recv(q[j].fd, x[k].p, (size_t)x[k].left, MSG_DONTWAIT);
					if (n < 0 && (errno == EAGAIN || errno == EINTR)) break;
					if (n <= 0) {
						free(q);
						free(x);
						return 1;
					}
					x[k].p += n;
					x[k].left -= n;
					break; /* streams are ordered: only the first pending op of this peer and direction */
				}
			}
		}
	}
	free(q);
	free(x);
	return 0;
}

static int sock_allgather(void *user, const double *send, double *recv, long count) {
	const int P = g_pinc.nranks, me = g_pinc.rank;
	long bytes = count * (long)sizeof(double);
	memcpy(recv + (long)me * count, send, bytes);
	if (P == 1) return 0;
	int *sp = malloc(P * sizeof(int)), *rp = malloc(P * sizeof(int));
	const void **sb = malloc(P * sizeof(void *));
	void **rb = malloc(P * sizeof(void *));
	long *nb = malloc(P * sizeof(long));
	int n = 0;
	for (int r = 0; r < P; r++) {
		if (r == me) continue;
		sp[n] = rp[n] = r;
		sb[n] = send;
		rb[n] = recv + (long)r * count;
		nb[n] = bytes;
		n++;
	}
	int rc = sock_exchange(user, n, sp, sb, nb, rp, rb, nb);
	free(sp);
	free(rp);
	free(sb);
	free(rb);
	free(nb);
	return rc;
}

/* sum in rank order 0..P-1 on every rank: the same result everywhere */
static int sock_allreduce_sum(void *user, double *buf, long count) {
	const int P = g_pinc.nranks;
	double *all = malloc((size_t)P * count * sizeof(double));
	if (!all) return 1;
	int rc = sock_allgather(user, buf, all, count);
	if (!rc)
		for (long i = 0; i < count; i++) {
			double s = 0;
			for (int r = 0; r < P; r++) s += all[(long)r * count + i];
			buf[i] = s;
		}
	free(all);
	return rc;
}

/* ---------------------------------------------------------- rendezvous -- */
typedef struct {
	unsigned magic;
	int rank, size;
	unsigned short port;
	unsigned char addr[4];
} Hello;
#define PINC_BOOT_MAGIC 0x50494e43u

static void rendezvous(int useHost) {
	const int P = g_pinc.nranks, me = g_pinc.rank;
	const char *addrs[] = {"PINC_MASTER_ADDR", "MASTER_ADDR", NULL};
	const char *host = env_first(addrs);
	if (!host) host = "127.0.0.1";
	unsigned short port = 29533;
	if (getenv("PINC_MASTER_PORT") && *getenv("PINC_MASTER_PORT")) port = (unsigned short)atoi(getenv("PINC_MASTER_PORT"));
	else if (getenv("MASTER_PORT") && *getenv("MASTER_PORT")) port = (unsigned short)(atoi(getenv("MASTER_PORT")) + 1);
	double tmo = getenv("PINC_BOOT_TIMEOUT") ? atof(getenv("PINC_BOOT_TIMEOUT")) : 120.0;
	double deadline = now_s() + tmo;
	g_nPeer = P;
	g_peer = malloc(P * sizeof(int));
	for (int r = 0; r < P; r++) g_peer[r] = -1;
	/* ranks > 0 listen for the mesh links of higher ranks */
	int meshL = -1;
	unsigned short meshPort = 0;
	if (useHost && me > 0) meshL = listen_on(0, &meshPort);
	Hello *tab = calloc(P, sizeof(Hello));
	unsigned char id[PINC_COMM_ID_BYTES];
	if (me == 0) {
		int lfd = listen_on(port, NULL);
		for (int k = 1; k < P; k++) {
			struct sockaddr_in a;
			socklen_t len = sizeof(a);
			int fd = accept_by(lfd, deadline, "rendezvous");
			Hello h;
			recv_all(fd, &h, sizeof(h), "rendezvous hello");
			if (h.magic != PINC_BOOT_MAGIC || h.size != P || h.rank <= 0 || h.rank >= P || g_peer[h.rank] >= 0)
				msg(ERROR | ALL, "[pinc rank 0] rendezvous: rank %d of %d does not fit a world of %d", h.rank, h.size, P);
			getpeername(fd, (struct sockaddr *)&a, &len);
			memcpy(h.addr, &a.sin_addr.s_addr, 4);
			tab[h.rank] = h;
			g_peer[h.rank] = fd;
		}
		close(lfd);
		if (useHost)
			for (int r = 1; r < P; r++) send_all(g_peer[r], tab, P * sizeof(Hello), "rendezvous table");
		else {
			pinc_check(pinc_hip_comm_unique_id(id), "RCCL unique id");
			for (int r = 1; r < P; r++) send_all(g_peer[r], id, sizeof(id), "RCCL id");
		}
	} else {
		int fd = connect_by(host, port, deadline, "rendezvous");
		Hello h = {PINC_BOOT_MAGIC, me, P, meshPort, {0, 0, 0, 0}};
		send_all(fd, &h, sizeof(h), "rendezvous hello");
		g_peer[0] = fd;
		if (useHost) recv_all(fd, tab, P * sizeof(Hello), "rendezvous table");
		else recv_all(fd, id, sizeof(id), "RCCL id");
	}
	if (useHost && me > 0) {
		/* connect to every lower rank > 0, then accept every higher one */
		for (int r = 1; r < me; r++) {
			char ip[INET_ADDRSTRLEN];
			inet_ntop(AF_INET, tab[r].addr, ip, sizeof(ip));
			int fd = connect_by(ip, tab[r].port, deadline, "mesh");
			send_all(fd, &me, sizeof(me), "mesh hello");
			g_peer[r] = fd;
		}
		for (int k = me + 1; k < P; k++) {
			int fd = accept_by(meshL, deadline, "mesh");
			int r = -1;
			recv_all(fd, &r, sizeof(r), "mesh hello");
			if (r <= me || r >= P || g_peer[r] >= 0) msg(ERROR | ALL, "[pinc rank %d] mesh: unexpected rank %d", me, r);
			g_peer[r] = fd;
		}
		close(meshL);
	}
	free(tab);
	if (useHost) {
		for (int r = 0; r < P; r++)
			if (g_peer[r] >= 0) fcntl(g_peer[r], F_SETFL, fcntl(g_peer[r], F_GETFL) | O_NONBLOCK);
		pinc_host_transport_t t = {sock_exchange, sock_allgather, sock_allreduce_sum, NULL};
		pinc_set_host_transport(&t);
		return;
	}
	for (int r = 0; r < P; r++)
		if (g_peer[r] >= 0) close(g_peer[r]);
	free(g_peer);
	g_peer = NULL;
	g_nPeer = 0;
	pinc_check(pinc_hip_comm_init(&g_pinc.comm, id, P, me), "RCCL communicator");
}

static void boot_close(void) {
	for (int r = 0; r < g_nPeer; r++)
		if (g_peer && g_peer[r] >= 0) close(g_peer[r]);
	free(g_peer);
	g_peer = NULL;
	g_nPeer = 0;
}

int pinc_boot_world(void) {
	if (g_booted) return g_pinc.nranks;
	g_booted = 1;
	if (g_configured || g_pinc.initialised) {
		/* the PincSim API (or an earlier call) configured the world */
		pinc_ctx_init();
		return g_pinc.nranks;
	}
	int rank, size, local;
	pinc_launcher_env(&rank, &size, &local);
	const char *tr = getenv("PINC_TRANSPORT");
	int useHost = tr && !strcmp(tr, "host");
	if (tr && *tr && !useHost && strcmp(tr, "rccl"))
		msg(ERROR | ALL, "PINC_TRANSPORT=%s (rccl or host)", tr);
	g_pinc.rank = rank;
	g_pinc.nranks = size;
	if (getenv("PINC_DEVICE") && *getenv("PINC_DEVICE")) {
		g_pinc.device = atoi(getenv("PINC_DEVICE"));
	} else if (useHost) {
		g_pinc.device = 0; /* several ranks share one GPU */
	} else {
		int n = 0;
		if (pinc_hip_device_count(&n) || n < 1) msg(ERROR | ALL, "no HIP device (%s)", pinc_hip_error_string());
		g_pinc.device = local % n;
	}
	pinc_ctx_init();
	if (size > 1) {
		rendezvous(useHost);
		atexit(boot_close);
	}
	return size;
}

/* Self-check of the TCP host transport without a GPU (tests/test_boot_cpu.py
 * runs it in `size` processes): rank and size as given, the rendezvous and
 * mesh of PINC_TRANSPORT=host, then an exchange with the slab neighbours
 * (pinc_ext_halo's pattern, ops paired as for two slabs), an allgather and an
 * allreduce of known values.  Returns 0 if every value arrived. */
int pinc_host_mesh_selftest(int rank, int size) {
	g_pinc.rank = rank;
	g_pinc.nranks = size;
	rendezvous(1);
	int bad = 0;
	const int up = (rank + 1) % size, dn = (rank - 1 + size) % size;
	enum { N = 100000 };
	double *a = malloc(N * sizeof(double)), *b = malloc(N * sizeof(double));
	double *ra = malloc(N * sizeof(double)), *rb = malloc(N * sizeof(double));
	for (int i = 0; i < N; i++) {
		a[i] = rank * 1e6 + i;      /* goes up */
		b[i] = -(rank * 1e6 + i);   /* goes down */
	}
	int sp[2] = {up, dn}, rp[2] = {dn, up};
	const void *sb[2] = {a, b};
	void *rbuf[2] = {ra, rb};
	long nb[2] = {N * (long)sizeof(double), N * (long)sizeof(double)};
	if (sock_exchange(NULL, 2, sp, sb, nb, rp, rbuf, nb)) bad |= 1;
	for (int i = 0; i < N; i++) {
		if (ra[i] != dn * 1e6 + i) bad |= 2;    /* what the lower rank sent up */
		if (rb[i] != -(up * 1e6 + i)) bad |= 4; /* what the upper rank sent down */
	}
	double v[3] = {rank, 1.0, rank * rank};
	double *all = malloc(3 * size * sizeof(double));
	if (sock_allgather(NULL, v, all, 3)) bad |= 8;
	for (int r = 0; r < size; r++)
		if (all[3 * r] != r || all[3 * r + 1] != 1.0 || all[3 * r + 2] != r * r) bad |= 16;
	if (sock_allreduce_sum(NULL, v, 3)) bad |= 32;
	if (v[0] != size * (size - 1) / 2.0 || v[1] != size) bad |= 64;
	free(a);
	free(b);
	free(ra);
	free(rb);
	free(all);
	boot_close();
	return bad;
}
