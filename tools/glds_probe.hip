// probe: LDS destination of global_load_lds for 4-, 12- and 16-byte pieces
// (which LDS bytes lane l writes), printed as the source dword index found
// at each LDS dword
#include <hip/hip_runtime.h>
#include <cstdio>
#define KDEF(SZ) \
__global__ void k##SZ(const unsigned *src, unsigned *out) { \
	__shared__ unsigned buf[1024]; \
	for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0xffffffffu; \
	__syncthreads(); \
	const char *g = (const char *)src + threadIdx.x * SZ; \
	__builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g, \
	                                 (__attribute__((address_space(3))) void *)buf, SZ, 0, 0); \
	__syncthreads(); \
	for (int i = threadIdx.x; i < 1024; i += 64) out[i] = buf[i]; \
}
KDEF(4) KDEF(12) KDEF(16)
// 16-byte pieces from 8-byte aligned sources (lane l reads dwords 2l+2..2l+5)
__global__ void k16u(const unsigned *src, unsigned *out) {
	__shared__ unsigned buf[1024];
	for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0xffffffffu;
	__syncthreads();
	const char *g = (const char *)src + 8 + threadIdx.x * 8;
	__builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
	                                 (__attribute__((address_space(3))) void *)buf, 16, 0, 0);
	__syncthreads();
	for (int i = threadIdx.x; i < 1024; i += 64) out[i] = buf[i];
}
#if 0
__global__ void k(const unsigned *src, unsigned *out) {
	__shared__ unsigned buf[1024];
	for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0xffffffffu;
	__syncthreads();
	const char *g = (const char *)src + threadIdx.x * SZ;
	__builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
	                                 (__attribute__((address_space(3))) void *)buf, SZ, 0, 0);
	__syncthreads();
	for (int i = threadIdx.x; i < 1024; i += 64) out[i] = buf[i];
}
#endif
int main() {
	unsigned h[2048], *ds, *dout;
	for (int i = 0; i < 2048; i++) h[i] = i;
	hipMalloc(&ds, sizeof(h));
	hipMalloc(&dout, 4096);
	hipMemcpy(ds, h, sizeof(h), hipMemcpyHostToDevice);
	unsigned o[1024];
#define RUN(SZ)                                                              \
	hipLaunchKernelGGL(k##SZ, dim3(1), dim3(64), 0, 0, ds, dout);           \
	hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost);                         \
	printf("size %d:", SZ);                                                  \
	for (int i = 0; i < 72; i++) printf(" %d", o[i] == 0xffffffffu ? -1 : (int)o[i]); \
	printf(" ... last written dword %d\n", [&] { int l = -1; for (int i = 0; i < 1024; i++) if (o[i] != 0xffffffffu) l = i; return l; }());
	RUN(4) RUN(12) RUN(16)
	hipLaunchKernelGGL(k16u, dim3(1), dim3(64), 0, 0, ds, dout);
	hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost);
	printf("size 16 from src+8+8l:");
	for (int i = 0; i < 24; i++) printf(" %d", o[i] == 0xffffffffu ? -1 : (int)o[i]);
	printf("\n");
	return 0;
}
