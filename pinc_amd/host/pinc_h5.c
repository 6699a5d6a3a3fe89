/*
 * pinc_h5.c -- the reference's HDF5 output files, written from the device
 * state (output formats for parity tooling).
 *
 *   gOpenH5/gWriteH5/gCloseH5   grid.c:1161-1270: <prefix>_<name>.grid.h5,
 *                               one dataset "/n=%.1f" per write, dims
 *                               [N_z..N_x, nValues] (true nodes only, global
 *                               frame), file attributes "Axis denormalization
 *                               factor" and "Quantity denormalization factor"
 *   pOpenH5/pWriteH5/pCloseH5   population.c:497-651: <prefix>_<name>.pop.h5,
 *                               groups /pos/specie s and /vel/specie s,
 *                               datasets "n=%.1f" [nParticles, nDims] in the
 *                               global frame, "Position/Velocity
 *                               denormalization factor" attributes
 *   xyOpenH5/xyCreateDataset/   io.c:603-734: extendible [n, 2] datasets,
 *   xyWrite/xyCloseH5           one (x, reduced y) row appended per write
 *   pCreateEnergyDatasets,      population.c:658-698: /energy/{potential,
 *   pWriteEnergy                kinetic}/{total,specie s}
 *
 * The reference writes through parallel HDF5 (MPI-IO hyperslabs, collective
 * transfers).  Here rank 0 writes the whole dataset with serial HDF5 after
 * an all-gather of the ranks' true nodes / particles over the library's
 * collectives (RCCL or the host transport); every rank ends with the same
 * file content the reference produces.  With the z-slab decomposition the
 * ranks' slabs are consecutive blocks of the file's C-order array.
 *
 * libhdf5 is loaded at run time (dlopen), so the hot path does not depend
 * on it: PINC_HDF5_LIB, else libhdf5.so / libhdf5_serial.so on the loader
 * path, else /opt/conda/lib/libhdf5.so.  A missing library is an error only
 * when output is requested.  The binding covers the HDF5 1.10 ABI (hid_t is
 * int64).
 */
#define _GNU_SOURCE
#include "pinc_internal.h"
#include <dlfcn.h>
#include <stdint.h>
#include <sys/stat.h>

typedef int64_t hid_t;
typedef unsigned long long hsize_t;
typedef int herr_t;
typedef int htri_t;
#define H5P_DEFAULT ((hid_t)0)
#define H5S_ALL ((hid_t)0)
#define H5S_SELECT_SET 0
#define H5F_ACC_RDONLY 0x0000u
#define H5F_ACC_RDWR 0x0001u
#define H5F_ACC_EXCL 0x0004u
#define H5S_UNLIMITED ((hsize_t)(-1))

static struct {
	void *lib;
	herr_t (*open)(void);
	hid_t (*Fcreate)(const char *, unsigned, hid_t, hid_t);
	hid_t (*Fopen)(const char *, unsigned, hid_t);
	herr_t (*Fclose)(hid_t);
	hid_t (*Screate_simple)(int, const hsize_t *, const hsize_t *);
	herr_t (*Sselect_hyperslab)(hid_t, int, const hsize_t *, const hsize_t *, const hsize_t *, const hsize_t *);
	int (*Sget_simple_extent_dims)(hid_t, hsize_t *, hsize_t *);
	herr_t (*Sclose)(hid_t);
	hid_t (*Dcreate2)(hid_t, const char *, hid_t, hid_t, hid_t, hid_t, hid_t);
	hid_t (*Dopen2)(hid_t, const char *, hid_t);
	herr_t (*Dwrite)(hid_t, hid_t, hid_t, hid_t, hid_t, const void *);
	herr_t (*Dread)(hid_t, hid_t, hid_t, hid_t, hid_t, void *);
	hid_t (*Dget_space)(hid_t);
	herr_t (*Dset_extent)(hid_t, const hsize_t *);
	herr_t (*Dclose)(hid_t);
	hid_t (*Pcreate)(hid_t);
	herr_t (*Pset_chunk)(hid_t, int, const hsize_t *);
	herr_t (*Pclose)(hid_t);
	hid_t (*Gcreate2)(hid_t, const char *, hid_t, hid_t, hid_t);
	herr_t (*Gclose)(hid_t);
	htri_t (*Lexists)(hid_t, const char *, hid_t);
	hid_t (*Acreate2)(hid_t, const char *, hid_t, hid_t, hid_t, hid_t);
	hid_t (*Aopen)(hid_t, const char *, hid_t);
	htri_t (*Aexists)(hid_t, const char *);
	herr_t (*Adelete)(hid_t, const char *);
	herr_t (*Awrite)(hid_t, hid_t, const void *);
	herr_t (*Aread)(hid_t, hid_t, void *);
	herr_t (*Aclose)(hid_t);
	hid_t *f64le, *nativeDouble, *clsDatasetCreate;
} H;

static void *sym(const char *name) {
	void *p = dlsym(H.lib, name);
	if (!p) msg(ERROR, "HDF5 output: symbol %s missing in the loaded libhdf5", name);
	return p;
}

static void h5_load(void) {
	if (H.lib) return;
	const char *cand[] = {getenv("PINC_HDF5_LIB"), "libhdf5.so", "libhdf5_serial.so", "/opt/conda/lib/libhdf5.so"};
	for (int i = 0; i < 4 && !H.lib; i++)
		if (cand[i] && *cand[i]) H.lib = dlopen(cand[i], RTLD_NOW | RTLD_LOCAL);
	if (!H.lib) msg(ERROR, "HDF5 output requested but no libhdf5 could be loaded (set PINC_HDF5_LIB)");
#define S(f, n) *(void **)&H.f = sym(n)
	S(open, "H5open");
	S(Fcreate, "H5Fcreate");
	S(Fopen, "H5Fopen");
	S(Fclose, "H5Fclose");
	S(Screate_simple, "H5Screate_simple");
	S(Sselect_hyperslab, "H5Sselect_hyperslab");
	S(Sget_simple_extent_dims, "H5Sget_simple_extent_dims");
	S(Sclose, "H5Sclose");
	S(Dcreate2, "H5Dcreate2");
	S(Dopen2, "H5Dopen2");
	S(Dwrite, "H5Dwrite");
	S(Dread, "H5Dread");
	S(Dget_space, "H5Dget_space");
	S(Dset_extent, "H5Dset_extent");
	S(Dclose, "H5Dclose");
	S(Pcreate, "H5Pcreate");
	S(Pset_chunk, "H5Pset_chunk");
	S(Pclose, "H5Pclose");
	S(Gcreate2, "H5Gcreate2");
	S(Gclose, "H5Gclose");
	S(Lexists, "H5Lexists");
	S(Acreate2, "H5Acreate2");
	S(Aopen, "H5Aopen");
	S(Aexists, "H5Aexists");
	S(Adelete, "H5Adelete");
	S(Awrite, "H5Awrite");
	S(Aread, "H5Aread");
	S(Aclose, "H5Aclose");
	S(f64le, "H5T_IEEE_F64LE_g");
	S(nativeDouble, "H5T_NATIVE_DOUBLE_g");
	S(clsDatasetCreate, "H5P_CLS_DATASET_CREATE_ID_g");
#undef S
	if (H.open() < 0) msg(ERROR, "H5open failed");
}

static void h5ok(long rc, const char *what) {
	if (rc < 0) msg(ERROR, "HDF5 output: %s failed", what);
}

/* ------------------------------------------------------------ helpers -- */

/* mkdir -p of the file's parent folders (io.c makePath) */
static void make_parent(const char *path) {
	char *p = strdup(path);
	for (char *c = p + 1; *c; c++)
		if (*c == '/') {
			*c = 0;
			mkdir(p, 0775);
			*c = '/';
		}
	free(p);
}

/* openH5File (io.c:566-602): <files:output><sep><fName>.<ext>.h5, opened
 * read-write if it exists, else created.  Rank 0 only (serial HDF5). */
static hid_t open_file(const dictionary *ini, const char *fName, const char *ext) {
	h5_load();
	char *pre = iniGetStr(ini, "files:output");
	size_t L = strlen(pre);
	const char *sep = "";
	if (!strcmp(pre, ".")) sep = "/";
	else if (L > 0 && pre[L - 1] != '/') sep = "_";
	size_t n = L + strlen(sep) + strlen(fName) + strlen(ext) + 8;
	char *name = malloc(n);
	snprintf(name, n, "%s%s%s.%s.h5", pre, sep, fName, ext);
	free(pre);
	hid_t f = -1;
	if (g_pinc.rank == 0) {
		make_parent(name);
		FILE *fh = fopen(name, "r");
		if (fh) {
			fclose(fh);
			f = H.Fopen(name, H5F_ACC_RDWR, H5P_DEFAULT);
		} else {
			f = H.Fcreate(name, H5F_ACC_EXCL, H5P_DEFAULT, H5P_DEFAULT);
		}
		if (f < 0) msg(ERROR, "could not open or create %s", name);
	}
	free(name);
	return f;
}

/* setH5Attr (io.c:604-627) */
static void set_attr(hid_t h5, const char *name, const double *value, int size) {
	if (h5 < 0) return;
	if (H.Aexists(h5, name) > 0) {
		msg(WARNING, "overwriting attribute \"%s\"", name);
		H.Adelete(h5, name);
	}
	hsize_t n = (hsize_t)size;
	hid_t sp = H.Screate_simple(1, &n, NULL);
	hid_t a = H.Acreate2(h5, name, *H.f64le, sp, H5P_DEFAULT, H5P_DEFAULT);
	h5ok(a, name);
	h5ok(H.Awrite(a, *H.nativeDouble, value), name);
	H.Aclose(a);
	H.Sclose(sp);
}

/* createH5Group (io.c:629-649): the parent groups of a dataset path */
static void make_groups(hid_t h5, const char *name) {
	char *s = strdup(name);
	for (char *c = s + 1; *c; c++)
		if (*c == '/') {
			*c = 0;
			if (H.Lexists(h5, s, H5P_DEFAULT) <= 0) H.Gclose(H.Gcreate2(h5, s, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
			*c = '/';
		}
	free(s);
}

static void write_dataset(hid_t h5, const char *name, int rank, const hsize_t *dims, const double *data) {
	/* main.c writes rho twice per step under one name (main.c:228 and 270):
	 * the reference's second H5Dcreate fails and the file keeps the first
	 * write; so here, without the error stack */
	if (H.Lexists(h5, name, H5P_DEFAULT) > 0) {
		static int warned = 0;
		if (!warned++)
			msg(WARNING, "HDF5 output: dataset %s exists (main.c:228,270 write rho twice per step); the first "
			             "write is kept, as the reference's H5Dcreate leaves it", name);
		return;
	}
	hid_t sp = H.Screate_simple(rank, dims, NULL);
	hid_t d = H.Dcreate2(h5, name, *H.f64le, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
	if (d < 0) msg(ERROR, "HDF5 output: cannot create dataset %s (exists already?)", name);
	h5ok(H.Dwrite(d, *H.nativeDouble, H5S_ALL, H5S_ALL, H5P_DEFAULT, data), name);
	H.Dclose(d);
	H.Sclose(sp);
}

/* every rank's `n` doubles, concatenated in rank order (rank 0 keeps them;
 * all ranks take part).  n may differ between ranks. */
static double *gather_host(const double *local, long n, long *total) {
	int P = g_pinc.nranks;
	if (P == 1) {
		*total = n;
		double *out = malloc((n > 0 ? n : 1) * sizeof(double));
		memcpy(out, local, n * sizeof(double));
		return out;
	}
	/* counts: each rank fills its slot, summed over ranks */
	double *cnt = NULL;
	pinc_check(pinc_hip_malloc((void **)&cnt, P * sizeof(double)), "h5 gather");
	double *hc = calloc(P, sizeof(double));
	hc[g_pinc.rank] = (double)n;
	pinc_check(pinc_hip_h2d(cnt, hc, P * sizeof(double), g_pinc.stream), "h5 gather");
	pinc_comm_allreduce_sum(cnt, P, "h5 counts");
	pinc_check(pinc_hip_d2h(hc, cnt, P * sizeof(double), g_pinc.stream), "h5 gather");
	long mx = 1;
	*total = 0;
	for (int r = 0; r < P; r++) {
		long c = (long)hc[r];
		if (c > mx) mx = c;
		*total += c;
	}
	double *dsend = NULL, *drecv = NULL;
	pinc_check(pinc_hip_malloc((void **)&dsend, mx * sizeof(double)), "h5 gather");
	pinc_check(pinc_hip_malloc((void **)&drecv, (long)P * mx * sizeof(double)), "h5 gather");
	pinc_check(pinc_hip_h2d(dsend, local, n * sizeof(double), g_pinc.stream), "h5 gather");
	pinc_comm_allgather(dsend, drecv, mx, "h5 gather");
	double *all = malloc((long)P * mx * sizeof(double));
	pinc_check(pinc_hip_d2h(all, drecv, (long)P * mx * sizeof(double), g_pinc.stream), "h5 gather");
	double *out = malloc((*total > 0 ? *total : 1) * sizeof(double));
	long o = 0;
	for (int r = 0; r < P; r++) {
		long c = (long)hc[r];
		memcpy(out + o, all + (long)r * mx, c * sizeof(double));
		o += c;
	}
	free(all);
	free(hc);
	pinc_hip_free(cnt);
	pinc_hip_free(dsend);
	pinc_hip_free(drecv);
	return out;
}

/* --------------------------------------------------------------- grid -- */

void gOpenH5(const dictionary *ini, Grid *grid, const MpiInfo *mpiInfo, const Units *units, double denorm,
             const char *fName) {
	(void)mpiInfo;
	hid_t f = open_file(ini, fName, "grid");
	set_attr(f, "Axis denormalization factor", &units->length, 1);
	set_attr(f, "Quantity denormalization factor", &denorm, 1);
	grid->h5 = f;
}

void gWriteH5(const Grid *grid, const MpiInfo *mpiInfo, double n) {
	(void)mpiInfo;
	gSyncToHost((Grid *)grid);
	int rank = grid->rank, nd = rank - 1, nv = grid->size[0];
	const int *sz = grid->size, *ts = grid->trueSize, *g = grid->nGhostLayers;
	long nTrue = nv;
	for (int d = 1; d <= nd; d++) nTrue *= ts[d];
	/* true nodes in C order [z][y][x][v] (value fastest, as grid->val) */
	double *loc = malloc(nTrue * sizeof(double));
	long o = 0;
	int T[3] = {1, 1, 1}, Sz[3] = {1, 1, 1}, G[3] = {0, 0, 0};
	for (int d = 0; d < nd; d++) {
		T[d] = ts[d + 1];
		Sz[d] = sz[d + 1];
		G[d] = g[d + 1];
	}
	for (int k = 0; k < T[2]; k++)
		for (int j = 0; j < T[1]; j++)
			for (int i = 0; i < T[0]; i++) {
				long node = (i + G[0]) + (long)Sz[0] * ((j + G[1]) + (long)Sz[1] * (k + G[2]));
				for (int v = 0; v < nv; v++) loc[o++] = grid->val[node * nv + v];
			}
	long tot = 0;
	double *all = gather_host(loc, nTrue, &tot);
	free(loc);
	if (g_pinc.rank == 0) {
		/* file dims reversed (grid.c:1240-1250): slowest = last dimension,
		 * which carries the z-slab decomposition */
		hsize_t dims[4];
		for (int d = 0; d < nd; d++) dims[d] = (hsize_t)ts[rank - 1 - d];
		dims[0] *= (hsize_t)g_pinc.nranks;
		dims[nd] = (hsize_t)nv;
		char name[64];
		snprintf(name, sizeof(name), "/n=%.1f", n);
		write_dataset(grid->h5, name, rank, dims, all);
	}
	free(all);
}

void gCloseH5(Grid *grid) {
	if (grid->h5 > 0) H.Fclose(grid->h5);
	grid->h5 = -1;
}

/* --------------------------------------------------------- population -- */

void pOpenH5(const dictionary *ini, Population *pop, const Units *units, const char *fName) {
	hid_t f = open_file(ini, fName, "pop");
	if (f >= 0) {
		H.Gclose(H.Gcreate2(f, "/pos", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
		H.Gclose(H.Gcreate2(f, "/vel", H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
		char name[48];
		for (int s = 0; s < pop->nSpecies; s++) {
			snprintf(name, sizeof(name), "/pos/specie %i", s);
			H.Gclose(H.Gcreate2(f, name, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
			snprintf(name, sizeof(name), "/vel/specie %i", s);
			H.Gclose(H.Gcreate2(f, name, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
		}
	}
	pop->h5 = f;
	set_attr(f, "Position denormalization factor", &units->length, 1);
	set_attr(f, "Velocity denormalization factor", &units->velocity, 1);
}

void pWriteH5(Population *pop, const MpiInfo *mpiInfo, double posN, double velN) {
	pSyncToHost(pop);
	int nd = pop->nDims;
	for (int s = 0; s < pop->nSpecies; s++) {
		long np = pop->iStop[s] - pop->iStart[s];
		/* global frame (pToGlobalFrame, population.c:721-740) */
		double *pos = malloc((np > 0 ? np : 1) * nd * sizeof(double));
		for (long i = 0; i < np; i++)
			for (int d = 0; d < nd; d++)
				pos[i * nd + d] = pop->pos[(pop->iStart[s] + i) * nd + d] + mpiInfo->offset[d];
		long tp = 0, tv = 0;
		double *ap = gather_host(pos, np * nd, &tp);
		double *av = gather_host(pop->vel + pop->iStart[s] * nd, np * nd, &tv);
		free(pos);
		if (g_pinc.rank == 0) {
			if (tp) {
				hsize_t dims[2] = {(hsize_t)(tp / nd), (hsize_t)nd};
				char name[64];
				snprintf(name, sizeof(name), "/pos/specie %i/n=%.1f", s, posN);
				write_dataset(pop->h5, name, 2, dims, ap);
				snprintf(name, sizeof(name), "/vel/specie %i/n=%.1f", s, velN);
				write_dataset(pop->h5, name, 2, dims, av);
			} else {
				msg(WARNING, "No particles of specie %i to store in .h5-file", s);
			}
		}
		free(ap);
		free(av);
	}
}

void pCloseH5(Population *pop) {
	if (pop->h5 > 0) H.Fclose(pop->h5);
	pop->h5 = -1;
}

/* ------------------------------------------------------------ history -- */

long long xyOpenH5(const dictionary *ini, const char *fName) { return open_file(ini, fName, "xy"); }

void xyCreateDataset(long long h5, const char *name) {
	if (h5 < 0) return;
	make_groups(h5, name);
	hsize_t chunk[2] = {1, 2}, dims[2] = {0, 2}, mx[2] = {H5S_UNLIMITED, 2};
	hid_t pl = H.Pcreate(*H.clsDatasetCreate);
	H.Pset_chunk(pl, 2, chunk);
	hid_t sp = H.Screate_simple(2, dims, mx);
	hid_t d = H.Dcreate2(h5, name, *H.f64le, sp, H5P_DEFAULT, pl, H5P_DEFAULT);
	h5ok(d, name);
	H.Sclose(sp);
	H.Dclose(d);
	H.Pclose(pl);
}

/* xyWrite (io.c:685-730): y reduced over the ranks (sum or max), row
 * (x, y) appended */
void xyWrite(long long h5, const char *name, double x, double y, int op) {
	double yr = y;
	if (g_pinc.nranks > 1) {
		long tot = 0;
		double *all = gather_host(&y, 1, &tot);
		yr = all[0];
		for (long r = 1; r < tot; r++) yr = op == PINC_OP_MAX ? (all[r] > yr ? all[r] : yr) : yr + all[r];
		free(all);
	}
	if (g_pinc.rank != 0) return;
	hid_t d = H.Dopen2(h5, name, H5P_DEFAULT);
	h5ok(d, name);
	hid_t fs = H.Dget_space(d);
	hsize_t dims[2];
	H.Sget_simple_extent_dims(fs, dims, NULL);
	dims[0]++;
	h5ok(H.Dset_extent(d, dims), "extend");
	H.Sclose(fs);
	fs = H.Dget_space(d);
	hsize_t off[2] = {dims[0] - 1, 0}, cnt[2] = {1, 1}, blk[2] = {1, 2};
	H.Sselect_hyperslab(fs, H5S_SELECT_SET, off, NULL, cnt, blk);
	double row[2] = {x, yr};
	hid_t ms = H.Screate_simple(2, blk, NULL);
	h5ok(H.Dwrite(d, *H.nativeDouble, ms, fs, H5P_DEFAULT, row), name);
	H.Sclose(ms);
	H.Sclose(fs);
	H.Dclose(d);
}

void xyCloseH5(long long h5) {
	if (h5 > 0) H.Fclose(h5);
}

void pCreateEnergyDatasets(long long xy, Population *pop) {
	char name[64];
	xyCreateDataset(xy, "/energy/potential/total");
	xyCreateDataset(xy, "/energy/kinetic/total");
	for (int s = 0; s < pop->nSpecies; s++) {
		snprintf(name, sizeof(name), "/energy/potential/specie %i", s);
		xyCreateDataset(xy, name);
		snprintf(name, sizeof(name), "/energy/kinetic/specie %i", s);
		xyCreateDataset(xy, name);
	}
}

/* pop->kinEnergy / potEnergy hold this rank's values; summed over ranks */
void pWriteEnergy(long long xy, Population *pop, double x) {
	pinc_pop_settle(pop); /* a fused puAcc3D1KE's sums */
	char name[64];
	int ns = pop->nSpecies;
	xyWrite(xy, "/energy/potential/total", x, pop->potEnergy[ns], PINC_OP_SUM);
	xyWrite(xy, "/energy/kinetic/total", x, pop->kinEnergy[ns], PINC_OP_SUM);
	for (int s = 0; s < ns; s++) {
		snprintf(name, sizeof(name), "/energy/potential/specie %i", s);
		xyWrite(xy, name, x, pop->potEnergy[s], PINC_OP_SUM);
		snprintf(name, sizeof(name), "/energy/kinetic/specie %i", s);
		xyWrite(xy, name, x, pop->kinEnergy[s], PINC_OP_SUM);
	}
}

/* ------------------------------------------------- read-back (tests) -- */

/* the dataset `name` of an .h5 file into out (at most cap doubles); returns
 * the element count, or -1.  Reads double attribute `name` when isAttr. */
long pinc_h5_read(const char *path, const char *name, int isAttr, double *out, long cap) {
	h5_load();
	hid_t f = H.Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
	if (f < 0) return -1;
	long n = -1;
	if (isAttr) {
		hid_t a = H.Aopen(f, name, H5P_DEFAULT);
		if (a >= 0) {
			double buf[16];
			if (H.Aread(a, *H.nativeDouble, buf) >= 0) {
				n = 1;
				if (cap >= 1) out[0] = buf[0];
			}
			H.Aclose(a);
		}
	} else {
		hid_t d = H.Dopen2(f, name, H5P_DEFAULT);
		if (d >= 0) {
			hid_t sp = H.Dget_space(d);
			hsize_t dims[8];
			int r = H.Sget_simple_extent_dims(sp, dims, NULL);
			n = 1;
			for (int i = 0; i < r; i++) n *= (long)dims[i];
			if (n <= cap && H.Dread(d, *H.nativeDouble, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0) n = -1;
			H.Sclose(sp);
			H.Dclose(d);
		}
	}
	H.Fclose(f);
	return n;
}

/* a new .h5 file holding one dataset (fixtures for tests, e.g. an /Object
 * mask for objects:file); returns 0 or -1 */
int pinc_h5_write(const char *path, const char *name, int rank, const long *dims, const double *data) {
	h5_load();
	hid_t f = H.Fcreate(path, 0x0002u /* H5F_ACC_TRUNC */, H5P_DEFAULT, H5P_DEFAULT);
	if (f < 0) return -1;
	hsize_t d[8];
	for (int i = 0; i < rank && i < 8; i++) d[i] = (hsize_t)dims[i];
	make_groups(f, name);
	write_dataset(f, name, rank, d, data);
	H.Fclose(f);
	return 0;
}

/* dims of a dataset (up to 8), returns its rank or -1 */
int pinc_h5_dims(const char *path, const char *name, long *dimsOut) {
	h5_load();
	hid_t f = H.Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
	if (f < 0) return -1;
	int r = -1;
	hid_t d = H.Dopen2(f, name, H5P_DEFAULT);
	if (d >= 0) {
		hid_t sp = H.Dget_space(d);
		hsize_t dims[8];
		r = H.Sget_simple_extent_dims(sp, dims, NULL);
		for (int i = 0; i < r; i++) dimsOut[i] = (long)dims[i];
		H.Sclose(sp);
		H.Dclose(d);
	}
	H.Fclose(f);
	return r;
}

int pinc_h5_available(void) {
	if (H.lib) return 1;
	const char *cand[] = {getenv("PINC_HDF5_LIB"), "libhdf5.so", "libhdf5_serial.so", "/opt/conda/lib/libhdf5.so"};
	for (int i = 0; i < 4; i++)
		if (cand[i] && *cand[i]) {
			void *l = dlopen(cand[i], RTLD_NOW | RTLD_LOCAL);
			if (l) {
				dlclose(l);
				return 1;
			}
		}
	return 0;
}
