// runtime.hip -- device, memory, stream/event and RCCL plumbing behind the
// C ABI of include/pinc_hip.h.  The reference's MPI calls on the hot path
// (grid.c:390-401 halo Sendrecv, pusher.c:930-1025 migrant exchange,
// grid.c:744-745 / multigrid.c:1478 Allreduce) map onto the RCCL calls here,
// one process per GPU over xGMI.
#include "common.h"
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

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

extern "C" int pinc_hip_comm_init(void **comm, const unsigned char *id, int nranks, int rank) {
	ncclUniqueId u;
	memcpy(&u, id, sizeof(u));
	ncclComm_t c;
	ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
	if (r != ncclSuccess) return nccl_error(r, "ncclCommInitRank");
	*comm = (void *)c;
	return 0;
}

extern "C" int pinc_hip_comm_destroy(void *comm) {
	if (!comm) return 0;
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
	return 0;
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
	return 0;
}

extern "C" int pinc_hip_comm_allgather(void *comm, const double *send, double *recv, long count,
                                       void *stream) {
	ncclResult_t r = ncclAllGather(send, recv, count, ncclDouble, (ncclComm_t)comm, (hipStream_t)stream);
	if (r != ncclSuccess) return nccl_error(r, "allgather");
	return 0;
}

extern "C" int pinc_hip_comm_allreduce_sum(void *comm, const double *send, double *recv, long count,
                                           void *stream) {
	ncclResult_t r = ncclAllReduce(send, recv, count, ncclDouble, ncclSum, (ncclComm_t)comm,
	                               (hipStream_t)stream);
	if (r != ncclSuccess) return nccl_error(r, "allreduce");
	return 0;
}
