// runtime.hip -- device, memory, stream/event and RCCL plumbing behind the
// C ABI of include/pinc_hip.h.  The reference's MPI calls on the hot path
// (grid.c:390-401 halo Sendrecv, pusher.c:930-1025 migrant exchange,
// grid.c:744-745 / multigrid.c:1478 Allreduce) map onto the RCCL calls here,
// one process per GPU over xGMI.
#include "common.h"
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <atomic>
#include <mutex>
#include <thread>

namespace pinc {

static thread_local char g_err[512] = "";

int set_error(hipError_t e, const char *where) {
	snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
	return (int)e ? (int)e : -1;
}

int check_launch(const char *where) {
	hipError_t e = hipGetLastError();
	if (e != hipSuccess) return set_error(e, where);
	return 0;
}

static int nccl_error(ncclResult_t r, const char *where) {
	snprintf(g_err, sizeof(g_err), "%s: %s", where, ncclGetErrorString(r));
	return 1000 + (int)r;
}

}  // namespace pinc

using namespace pinc;

#define HIPCALL(expr, where)                                 \
	do {                                                     \
		hipError_t _e = (expr);                              \
		if (_e != hipSuccess) return set_error(_e, where);  \
	} while (0)

extern "C" const char *pinc_hip_error_string(void) { return g_err; }

extern "C" int pinc_hip_set_device(int dev) {
	HIPCALL(hipSetDevice(dev), "hipSetDevice");
	return 0;
}

extern "C" int pinc_hip_device_count(int *n) {
	HIPCALL(hipGetDeviceCount(n), "hipGetDeviceCount");
	return 0;
}

extern "C" int pinc_hip_stream_create(void **stream) {
	hipStream_t s;
	HIPCALL(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
	*stream = (void *)s;
	return 0;
}

extern "C" int pinc_hip_stream_destroy(void *stream) {
	HIPCALL(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
	return 0;
}

// stream capture into a replayable graph (a fixed launch sequence, e.g. one
// V-cycle): begin, end -> instantiated executable, launch, destroy
extern "C" int pinc_hip_capture_begin(void *stream) {
	HIPCALL(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
	return 0;
}

// the executable keeps its graph alive until both are destroyed together
struct PincGraph {
	hipGraph_t g;
	hipGraphExec_t e;
};

extern "C" int pinc_hip_capture_end(void *stream, void **exec) {
	hipGraph_t g = nullptr;
	HIPCALL(hipStreamEndCapture((hipStream_t)stream, &g), "hipStreamEndCapture");
	hipGraphExec_t e = nullptr;
	hipError_t r = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
	if (r != hipSuccess) {
		(void)hipGraphDestroy(g);
		HIPCALL(r, "hipGraphInstantiate");
	}
	PincGraph *pg = new PincGraph{g, e};
	*exec = (void *)pg;
	return 0;
}

extern "C" int pinc_hip_graph_launch(void *exec, void *stream) {
	HIPCALL(hipGraphLaunch(((PincGraph *)exec)->e, (hipStream_t)stream), "hipGraphLaunch");
	return 0;
}

extern "C" int pinc_hip_graph_destroy(void *exec) {
	if (!exec) return 0;
	PincGraph *pg = (PincGraph *)exec;
	hipError_t r1 = hipGraphExecDestroy(pg->e);
	hipError_t r2 = hipGraphDestroy(pg->g);
	delete pg;
	HIPCALL(r1, "hipGraphExecDestroy");
	HIPCALL(r2, "hipGraphDestroy");
	return 0;
}

extern "C" int pinc_hip_stream_sync(void *stream) {
	HIPCALL(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
	return 0;
}

extern "C" int pinc_hip_device_sync(void) {
	HIPCALL(hipDeviceSynchronize(), "hipDeviceSynchronize");
	return 0;
}

extern "C" int pinc_hip_malloc(void **ptr, unsigned long bytes) {
	if (bytes == 0) bytes = 16;
	HIPCALL(hipMalloc(ptr, bytes), "hipMalloc");
	return 0;
}

extern "C" int pinc_hip_free(void *ptr) {
	if (!ptr) return 0;
	HIPCALL(hipFree(ptr), "hipFree");
	return 0;
}

extern "C" int pinc_hip_memset(void *ptr, int value, unsigned long bytes, void *stream) {
	if (!bytes) return 0;
	HIPCALL(hipMemsetAsync(ptr, value, bytes, (hipStream_t)stream), "hipMemsetAsync");
	return 0;
}

extern "C" int pinc_hip_h2d(void *dst, const void *src, unsigned long bytes, void *stream) {
	if (!bytes) return 0;
	HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream), "h2d");
	HIPCALL(hipStreamSynchronize((hipStream_t)stream), "h2d sync");
	return 0;
}

extern "C" int pinc_hip_d2h(void *dst, const void *src, unsigned long bytes, void *stream) {
	if (!bytes) return 0;
	HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream), "d2h");
	HIPCALL(hipStreamSynchronize((hipStream_t)stream), "d2h sync");
	return 0;
}

extern "C" int pinc_hip_d2h_async(void *dst, const void *src, unsigned long bytes, void *stream) {
	if (!bytes) return 0;
	HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream), "d2h async");
	return 0;
}

extern "C" int pinc_hip_host_alloc(void **ptr, unsigned long bytes) {
	if (bytes == 0) bytes = 16;
	HIPCALL(hipHostMalloc(ptr, bytes, hipHostMallocDefault), "hipHostMalloc");
	return 0;
}

extern "C" int pinc_hip_host_free(void *ptr) {
	if (!ptr) return 0;
	HIPCALL(hipHostFree(ptr), "hipHostFree");
	return 0;
}

extern "C" int pinc_hip_event_sync(void *ev) {
	HIPCALL(hipEventSynchronize((hipEvent_t)ev), "hipEventSynchronize");
	return 0;
}

extern "C" int pinc_hip_d2d(void *dst, const void *src, unsigned long bytes, void *stream) {
	if (!bytes) return 0;
	HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream), "d2d");
	return 0;
}

extern "C" int pinc_hip_event_create(void **ev) {
	hipEvent_t e;
	HIPCALL(hipEventCreate(&e), "hipEventCreate");
	*ev = (void *)e;
	return 0;
}

extern "C" int pinc_hip_event_destroy(void *ev) {
	HIPCALL(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy");
	return 0;
}

extern "C" int pinc_hip_event_record(void *ev, void *stream) {
	HIPCALL(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "hipEventRecord");
	return 0;
}

extern "C" int pinc_hip_event_elapsed(float *ms, void *start, void *stop) {
	HIPCALL(hipEventSynchronize((hipEvent_t)stop), "hipEventSynchronize");
	HIPCALL(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop), "hipEventElapsedTime");
	return 0;
}

extern "C" int pinc_hip_mem_info(unsigned long *freeBytes, unsigned long *totalBytes) {
	size_t f = 0, t = 0;
	HIPCALL(hipMemGetInfo(&f, &t), "hipMemGetInfo");
	*freeBytes = f;
	*totalBytes = t;
	return 0;
}

// ----------------------------------------------------------------- RCCL ---
static_assert(sizeof(ncclUniqueId) == PINC_COMM_ID_BYTES, "ncclUniqueId size");

extern "C" int pinc_hip_comm_unique_id(unsigned char *id) {
	ncclUniqueId u;
	ncclResult_t r = ncclGetUniqueId(&u);
	if (r != ncclSuccess) return nccl_error(r, "ncclGetUniqueId");
	memcpy(id, &u, sizeof(u));
	return 0;
}

// Watchdog of the RCCL calls.  A collective whose peers never post the
// matching call (a rank that skipped or reordered one) does not fail in RCCL:
// the stream just never drains and the job hangs.  Every enqueued RCCL call
// records an event behind it; a host thread polls the newest one, and when
// the calls enqueued since the stream was last seen drained have not
// completed within PINC_COMM_TIMEOUT seconds (default 300, 0 = off), or
// RCCL reports an asynchronous error, it names the call, aborts the
// communicator (ncclCommAbort) and ends the process with exit status 3.
namespace {
struct CommWatch {
	std::mutex m;
	std::thread th;
	std::atomic<bool> stop{false};
	ncclComm_t comm = nullptr;
	static constexpr int kRing = 64;
	hipEvent_t ev[kRing];
	int latest = -1;
	bool armed = false;
	double t0 = 0, timeout = 300;
	long seq = 0, seqFirst = 0;
	char what[96] = "", whatFirst[96] = "";
	int rank = 0;
};
CommWatch *g_watch = nullptr;

double mono_s() {
	timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

[[noreturn]] void watch_fail(CommWatch *w, const char *why) {
	fprintf(stderr,
	        "[pinc rank %d] RCCL watchdog: %s; oldest pending call #%ld (%s), newest #%ld (%s); aborting the "
	        "communicator\n",
	        w->rank, why, w->seqFirst, w->whatFirst, w->seq, w->what);
	fflush(stderr);
	ncclCommAbort(w->comm);
	_exit(3);
}

void watch_loop(CommWatch *w) {
	while (!w->stop.load()) {
		usleep(100000);
		std::lock_guard<std::mutex> g(w->m);
		ncclResult_t ae = ncclSuccess;
		if (ncclCommGetAsyncError(w->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
			char b[160];
			snprintf(b, sizeof(b), "asynchronous error %s", ncclGetErrorString(ae));
			watch_fail(w, b);
		}
		if (!w->armed) continue;
		hipError_t q = hipEventQuery(w->ev[w->latest]);
		if (q == hipSuccess) {
			w->armed = false;
			continue;
		}
		if (q != hipErrorNotReady) watch_fail(w, hipGetErrorString(q));
		if (w->timeout > 0 && mono_s() - w->t0 > w->timeout) {
			char b[160];
			snprintf(b, sizeof(b), "no completion for %.0f s (PINC_COMM_TIMEOUT)", w->timeout);
			watch_fail(w, b);
		}
	}
}

thread_local char g_note[96] = "";

// after an RCCL call was enqueued on `stream`
int watch_mark(hipStream_t stream, const char *kind) {
	char what[200];
	snprintf(what, sizeof(what), "%s %s", kind, g_note);
	CommWatch *w = g_watch;
	if (!w) return 0;
	std::lock_guard<std::mutex> g(w->m);
	if (w->armed && hipEventQuery(w->ev[w->latest]) == hipSuccess) w->armed = false;
	const int idx = (w->latest + 1) % CommWatch::kRing;
	HIPCALL(hipEventRecord(w->ev[idx], stream), "watchdog event");
	w->latest = idx;
	w->seq++;
	snprintf(w->what, sizeof(w->what), "%s", what);
	if (!w->armed) {
		w->armed = true;
		w->t0 = mono_s();
		w->seqFirst = w->seq;
		snprintf(w->whatFirst, sizeof(w->whatFirst), "%s", what);
	}
	return 0;
}
}  // namespace

extern "C" int pinc_hip_comm_note(const char *what) {
	snprintf(g_note, sizeof(g_note), "%s", what ? what : "");
	return 0;
}

extern "C" int pinc_hip_comm_init(void **comm, const unsigned char *id, int nranks, int rank) {
	ncclUniqueId u;
	memcpy(&u, id, sizeof(u));
	ncclComm_t c;
	ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
	if (r != ncclSuccess) return nccl_error(r, "ncclCommInitRank");
	*comm = (void *)c;
	if (!g_watch) {
		CommWatch *w = new CommWatch;
		w->comm = c;
		w->rank = rank;
		if (const char *t = getenv("PINC_COMM_TIMEOUT")) w->timeout = atof(t);
		for (int i = 0; i < CommWatch::kRing; i++)
			HIPCALL(hipEventCreateWithFlags(&w->ev[i], hipEventDisableTiming), "watchdog events");
		w->th = std::thread(watch_loop, w);
		g_watch = w;
	}
	return 0;
}

extern "C" int pinc_hip_comm_destroy(void *comm) {
	if (!comm) return 0;
	if (g_watch && g_watch->comm == (ncclComm_t)comm) {
		g_watch->stop.store(true);
		g_watch->th.join();
		for (int i = 0; i < CommWatch::kRing; i++) hipEventDestroy(g_watch->ev[i]);
		delete g_watch;
		g_watch = nullptr;
	}
	ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
	if (r != ncclSuccess) return nccl_error(r, "ncclCommDestroy");
	return 0;
}

extern "C" int pinc_hip_comm_sendrecv(void *comm, const void *sendbuf, long sendBytes, int peerSend,
                                      void *recvbuf, long recvBytes, int peerRecv, void *stream) {
	ncclComm_t c = (ncclComm_t)comm;
	hipStream_t st = (hipStream_t)stream;
	ncclResult_t r = ncclGroupStart();
	if (r == ncclSuccess && sendBytes > 0) r = ncclSend(sendbuf, sendBytes, ncclUint8, peerSend, c, st);
	if (r == ncclSuccess && recvBytes > 0) r = ncclRecv(recvbuf, recvBytes, ncclUint8, peerRecv, c, st);
	ncclResult_t r2 = ncclGroupEnd();
	if (r != ncclSuccess) return nccl_error(r, "sendrecv");
	if (r2 != ncclSuccess) return nccl_error(r2, "sendrecv group");
	return watch_mark(st, "sendrecv");
}

extern "C" int pinc_hip_comm_exchange(void *comm, int nOps, const int *sendPeer, void *const *sendbuf,
                                      const long *sendBytes, const int *recvPeer, void *const *recvbuf,
                                      const long *recvBytes, void *stream) {
	ncclComm_t c = (ncclComm_t)comm;
	hipStream_t st = (hipStream_t)stream;
	ncclResult_t r = ncclGroupStart();
	for (int i = 0; i < nOps && r == ncclSuccess; i++) {
		if (sendBytes[i] > 0) r = ncclSend(sendbuf[i], sendBytes[i], ncclUint8, sendPeer[i], c, st);
		if (r == ncclSuccess && recvBytes[i] > 0)
			r = ncclRecv(recvbuf[i], recvBytes[i], ncclUint8, recvPeer[i], c, st);
	}
	ncclResult_t r2 = ncclGroupEnd();
	if (r != ncclSuccess) return nccl_error(r, "exchange");
	if (r2 != ncclSuccess) return nccl_error(r2, "exchange group");
	return watch_mark(st, "exchange");
}

extern "C" int pinc_hip_comm_allgather(void *comm, const double *send, double *recv, long count,
                                       void *stream) {
	ncclResult_t r = ncclAllGather(send, recv, count, ncclDouble, (ncclComm_t)comm, (hipStream_t)stream);
	if (r != ncclSuccess) return nccl_error(r, "allgather");
	return watch_mark((hipStream_t)stream, "allgather");
}

extern "C" int pinc_hip_comm_allreduce_sum(void *comm, const double *send, double *recv, long count,
                                           void *stream) {
	ncclResult_t r = ncclAllReduce(send, recv, count, ncclDouble, ncclSum, (ncclComm_t)comm,
	                               (hipStream_t)stream);
	if (r != ncclSuccess) return nccl_error(r, "allreduce");
	return watch_mark((hipStream_t)stream, "allreduce");
}

// ------------------------------------------------------------ test hook ---
// A kernel that occupies the stream for `seconds` of wall time (one lane
// polling s_memrealtime, 100 MHz, with s_sleep between polls), so that a test
// can hold an RCCL call behind it and watch the watchdog fire (or not).  The
// bound is the kernel's own: every launch ends by itself.
namespace {
__global__ void k_test_spin(unsigned long long ticks) {
	if (threadIdx.x != 0) return;
	const unsigned long long t0 = wall_clock64();
	while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

extern "C" int pinc_hip_test_spin(double seconds, void *stream) {
	if (!(seconds >= 0.0) || seconds > 30.0) return set_error(hipErrorInvalidValue, "test spin: 0..30 s");
	hipLaunchKernelGGL(k_test_spin, dim3(1), dim3(64), 0, (hipStream_t)stream,
	                   (unsigned long long)(seconds * 1e8));
	return check_launch("test spin");
}
