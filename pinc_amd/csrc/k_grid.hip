// k_grid.hip -- grid glue of the PINC timestep on MI355X (gfx950).
//   scale / zero           gMul / gZero                 grid.c:668-714
//   fold_self              gHaloOp(addSlice, FROMHALO)  grid.c:340-406 (self-periodic slab dim)
//   efield                 gFinDiff1st + TOHALO (grid.c:226-261, main.c:245-246); the
//                          caller's gMul(E,-1) negates
//   sum / dot / reduce     gSumTruegrid / gPotEnergy    grid.c:804-847, 1276-1321
// Reductions are two-stage with a fixed block count, so results are bitwise
// reproducible run to run (they differ from the reference's sequential sums
// only by summation order).
#include "common.h"

using namespace pinc;

namespace {

constexpr int kThreads = 256;
constexpr int kRedBlocks = 1024;

inline long ceil_div(long a, long b) { return (a + b - 1) / b; }
inline unsigned grid_for(long n, int per = 4) {
	long b = ceil_div(n, (long)kThreads * per);
	if (b < 1) b = 1;
	if (b > 262144) b = 262144;
	return (unsigned)b;
}

__global__ void k_fill(double *a, long n, double v) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		a[i] = v;
}

__global__ void k_scale(double *a, long n, double f) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		a[i] = a[i] * f;
}

__global__ void k_scale2(double *a, long n, double f1, double f2) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		a[i] = (a[i] * f1) * f2;
}

__global__ void k_sub_dev(double *a, long n, const double *mu) {
	double m = *mu;
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		a[i] = a[i] - m;
}

// linear extrapolation in time: phi <- 2 phi - prev, prev <- phi (the
// multigrid's initial guess from the last two solutions)
__global__ void k_extrapolate(double *__restrict__ phi, double *__restrict__ prev, long n) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		const double p = phi[i];
		phi[i] = 2.0 * p - prev[i];
		prev[i] = p;
	}
}

__global__ void k_lincomb(double *out, const double *x, double a, const double *y, double b, long n) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		out[i] = a * x[i] + b * y[i];
}

// plane p of a slab: plane size = product of the non-slab extents
__global__ void k_add_plane(double *dst, const double *src, long planeSize) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < planeSize; i += (long)gridDim.x * blockDim.x)
		dst[i] += src[i];
}

__global__ void k_copy(double *dst, const double *src, long n) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		dst[i] = src[i];
}

// one slab plane per blockIdx.y, the plane's nodes (x fastest) over
// blockIdx.x: 32-bit in-plane coordinates, no 64-bit division per node
// (same expression per component as k_efield)
template <int ND>
__global__ void k_efield_planes(const double *__restrict__ phi, pinc_geom_t g, double *__restrict__ E, double h) {
	const int sd = ND - 1;
	const int T0 = g.T[0], T1 = ND > 1 ? g.T[1] : 1;
	const unsigned ps = ND == 3 ? (unsigned)T0 * T1 : ND == 2 ? (unsigned)T0 : 1u;  // nodes per slab plane
	const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= ps) return;
	const int p = blockIdx.y;  // slab plane 0 .. nloc+1
	int c[3] = {0, 0, 0};
	if (ND == 3) {
		c[1] = (int)(i / (unsigned)T0);
		c[0] = (int)(i - (unsigned)c[1] * T0);
	} else if (ND == 2) {
		c[0] = (int)i;
	}
	const int Ts = g.T[sd];
	c[sd] = wrap(g.off + p - 1, Ts);
	const long gs[3] = {1, T0, (long)T0 * T1};
	long gi = 0;
#pragma unroll
	for (int d = 0; d < ND; d++) gi += (long)c[d] * gs[d];
	const long idx = (long)p * ps + i;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		const int Td = g.T[d];
		const long up = gi + (long)(wrap(c[d] + 1, Td) - c[d]) * gs[d];
		const long dn = gi + (long)(wrap(c[d] - 1, Td) - c[d]) * gs[d];
		E[idx * ND + d] = h * (phi[up] - phi[dn]);
	}
}

template <int ND>
__global__ void k_efield(const double *__restrict__ phi, pinc_geom_t g, double *__restrict__ E, double h) {
	// slab nodes: non-slab dims periodic [0,T), slab dim planes 0..nloc+1
	int T[3] = {g.T[0], g.T[1], g.T[2]};
	int sd = ND - 1;
	long ext[3];
	for (int d = 0; d < 3; d++) ext[d] = (d < ND) ? (d == sd ? g.nloc + 2 : T[d]) : 1;
	long n = ext[0] * ext[1] * ext[2];
	long gs[3] = {1, T[0], (long)T[0] * T[1]};
	for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
		int c[3];
		long r = idx;
		for (int d = 0; d < 3; d++) {
			c[d] = (int)(r % ext[d]);
			r /= ext[d];
		}
		// global coordinate of the slab plane (periodic)
		c[sd] = wrap(g.off + c[sd] - 1, T[sd]);
		long gi = 0;
		for (int d = 0; d < ND; d++) gi += (long)c[d] * gs[d];
#pragma unroll
		for (int d = 0; d < ND; d++) {
			long up = gi + (long)(wrap(c[d] + 1, T[d]) - c[d]) * gs[d];
			long dn = gi + (long)(wrap(c[d] - 1, T[d]) - c[d]) * gs[d];
			E[idx * ND + d] = h * (phi[up] - phi[dn]);
		}
	}
}

template <int ND>
__global__ void k_slab_from_global(double *__restrict__ slab, const double *__restrict__ glob,
                                   pinc_geom_t g, int nv) {
	int T[3] = {g.T[0], g.T[1], g.T[2]};
	int sd = ND - 1;
	long ext[3];
	for (int d = 0; d < 3; d++) ext[d] = (d < ND) ? (d == sd ? g.nloc + 2 : T[d]) : 1;
	long n = ext[0] * ext[1] * ext[2];
	long gs[3] = {1, T[0], (long)T[0] * T[1]};
	for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
		int c[3];
		long r = idx;
		for (int d = 0; d < 3; d++) {
			c[d] = (int)(r % ext[d]);
			r /= ext[d];
		}
		c[sd] = wrap(g.off + c[sd] - 1, T[sd]);
		long gi = 0;
		for (int d = 0; d < ND; d++) gi += (long)c[d] * gs[d];
		for (int v = 0; v < nv; v++) slab[idx * nv + v] = glob[gi * nv + v];
	}
}

__global__ __launch_bounds__(kThreads) void k_sum(const double *__restrict__ a,
                                                  const double *__restrict__ b, long n,
                                                  double *__restrict__ partial) {
	__shared__ double red[kThreads / 64];
	double s = 0.;
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
		s += b ? a[i] * b[i] : a[i];
	double t = block_sum(s, red);
	if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(kThreads) void k_reduce(const double *__restrict__ partial, int n,
                                                     double div, double *__restrict__ out) {
	__shared__ double red[kThreads / 64];
	double s = 0.;
	for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
	double t = block_sum(s, red);
	if (threadIdx.x == 0) *out = t / div;
}

inline unsigned red_blocks(long n) {
	long b = ceil_div(n, (long)kThreads * 8);
	if (b < 1) b = 1;
	if (b > kRedBlocks) b = kRedBlocks;
	return (unsigned)b;
}

}  // namespace

extern "C" int pinc_hip_zero(double *a, long n, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a, n, 0.0);
	return check_launch("zero");
}

extern "C" int pinc_hip_scale(double *a, long n, double f, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a, n, f);
	return check_launch("scale");
}

extern "C" int pinc_hip_scale2(double *a, long n, double f1, double f2, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_scale2, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a, n, f1, f2);
	return check_launch("scale2");
}

extern "C" int pinc_hip_sub_dev(double *a, long n, const double *mu, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_sub_dev, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a, n, mu);
	return check_launch("sub_dev");
}

extern "C" int pinc_hip_extrapolate(double *phi, double *prev, long n, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_extrapolate, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, phi, prev, n);
	return check_launch("extrapolate");
}

extern "C" int pinc_hip_lincomb(double *out, const double *x, double a, const double *y, double b, long n,
                                void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_lincomb, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, out, x, a, y, b, n);
	return check_launch("lincomb");
}

static long plane_size(const pinc_geom_t &g) {
	long p = 1;
	for (int d = 0; d < g.nd - 1; d++) p *= g.T[d];
	return p;
}

extern "C" int pinc_hip_fold_self(double *slab, pinc_geom_t g, void *stream) {
	long ps = plane_size(g);
	hipStream_t st = (hipStream_t)stream;
	// grid.c:392-402 with the slab sending to itself: first the upper ghost
	// plane is added into plane 1, then the lower ghost into plane nloc
	hipLaunchKernelGGL(k_add_plane, dim3(grid_for(ps)), dim3(kThreads), 0, st, slab + ps,
	                   slab + (long)(g.nloc + 1) * ps, ps);
	hipLaunchKernelGGL(k_add_plane, dim3(grid_for(ps)), dim3(kThreads), 0, st, slab + (long)g.nloc * ps, slab, ps);
	return check_launch("fold_self");
}

extern "C" int pinc_hip_add(double *a, const double *b, long n, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_add_plane, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a, b, n);
	return check_launch("add");
}

extern "C" int pinc_hip_slab_from_global(double *slab, const double *global, pinc_geom_t g, int nValues,
                                         void *stream) {
	long n = plane_size(g) * (g.nloc + 2);
	hipStream_t st = (hipStream_t)stream;
	if (g.nd == 3) hipLaunchKernelGGL(k_slab_from_global<3>, dim3(grid_for(n)), dim3(kThreads), 0, st, slab, global, g, nValues);
	else if (g.nd == 2) hipLaunchKernelGGL(k_slab_from_global<2>, dim3(grid_for(n)), dim3(kThreads), 0, st, slab, global, g, nValues);
	else hipLaunchKernelGGL(k_slab_from_global<1>, dim3(grid_for(n)), dim3(kThreads), 0, st, slab, global, g, nValues);
	return check_launch("slab_from_global");
}

extern "C" int pinc_hip_add_plane(double *slab, pinc_geom_t g, int plane, const double *in, void *stream) {
	long ps = plane_size(g);
	hipLaunchKernelGGL(k_add_plane, dim3(grid_for(ps)), dim3(kThreads), 0, (hipStream_t)stream,
	                   slab + (long)plane * ps, in, ps);
	return check_launch("add_plane");
}

extern "C" int pinc_hip_copy_plane(double *dst, const double *slab, pinc_geom_t g, int plane,
                                   int nValues, void *stream) {
	long ps = plane_size(g) * nValues;
	hipLaunchKernelGGL(k_copy, dim3(grid_for(ps)), dim3(kThreads), 0, (hipStream_t)stream, dst,
	                   slab + (long)plane * ps, ps);
	return check_launch("copy_plane");
}

// h = 0.5: gFinDiff1st (grid.c:226-261); h = -0.5: the same followed by
// gMul(E, -1) (main.c:247), bit for bit (the negation and the halving are
// exact, and IEEE rounding is symmetric in the sign)
extern "C" int pinc_hip_efield_scaled(const double *phi, pinc_geom_t g, double *E, double h, void *stream) {
	if (h != 0.5 && h != -0.5) return set_error(hipErrorInvalidValue, "efield: h must be 0.5 or -0.5");
	long n = plane_size(g) * (g.nloc + 2);
	hipStream_t st = (hipStream_t)stream;
	if (plane_size(g) < (1L << 31) && g.nloc + 2 <= 65535) {
		const dim3 grid((unsigned)ceil_div(plane_size(g), kThreads), (unsigned)(g.nloc + 2));
		if (g.nd == 3) hipLaunchKernelGGL(k_efield_planes<3>, grid, dim3(kThreads), 0, st, phi, g, E, h);
		else if (g.nd == 2) hipLaunchKernelGGL(k_efield_planes<2>, grid, dim3(kThreads), 0, st, phi, g, E, h);
		else hipLaunchKernelGGL(k_efield_planes<1>, grid, dim3(kThreads), 0, st, phi, g, E, h);
		return check_launch("efield");
	}
	if (g.nd == 3) hipLaunchKernelGGL(k_efield<3>, dim3(grid_for(n)), dim3(kThreads), 0, st, phi, g, E, h);
	else if (g.nd == 2) hipLaunchKernelGGL(k_efield<2>, dim3(grid_for(n)), dim3(kThreads), 0, st, phi, g, E, h);
	else hipLaunchKernelGGL(k_efield<1>, dim3(grid_for(n)), dim3(kThreads), 0, st, phi, g, E, h);
	return check_launch("efield");
}

extern "C" int pinc_hip_efield(const double *phi, pinc_geom_t g, double *E, void *stream) {
	return pinc_hip_efield_scaled(phi, g, E, 0.5, stream);
}

extern "C" int pinc_hip_reduce(const double *partial, int n, double div, double *out, void *stream) {
	hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, partial, n, div, out);
	return check_launch("reduce");
}

extern "C" int pinc_hip_sum(const double *a, long n, double *partial, double *out, void *stream) {
	unsigned nb = red_blocks(n);
	hipLaunchKernelGGL(k_sum, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, a, (const double *)nullptr, n, partial);
	return pinc_hip_reduce(partial, (int)nb, 1.0, out, stream);
}

extern "C" int pinc_hip_sum_div(const double *a, long n, double div, double *partial, double *out,
                                void *stream) {
	unsigned nb = red_blocks(n);
	hipLaunchKernelGGL(k_sum, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, a, (const double *)nullptr, n, partial);
	return pinc_hip_reduce(partial, (int)nb, div, out, stream);
}

extern "C" int pinc_hip_dot(const double *a, const double *b, long n, double *partial, double *out, void *stream) {
	unsigned nb = red_blocks(n);
	hipLaunchKernelGGL(k_sum, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, a, b, n, partial);
	return pinc_hip_reduce(partial, (int)nb, 1.0, out, stream);
}
