/*
 * pinc_hip.h -- C ABI of the MI355X kernel library (libpinc_hip.so).
 *
 * Plain C: pointers, sizes and small POD structs only; no HIP or torch types
 * cross this boundary (streams are opaque void*).  Every entry point returns
 * 0 on success or a nonzero HIP/RCCL error code; pinc_hip_error_string()
 * describes the last failure.  The host operator surface (include/pinc.h)
 * is built on these calls; each entry cites the reference loop it replaces.
 *
 * Device data layout (DESIGN.md "Layout"):
 *   particles  SoA per component, species s in [iStart[s], iStart[s+1]) with
 *              live particles [iStart[s], iStop[s]) -- the reference's
 *              Population ranges (core.h:72-86) with x,y,z,vx,vy,vz split.
 *              Positions are in the reference's local frame (true nodes at
 *              1..T, ghosts 0 and T+1).
 *   slab grid  the decomposed (last) dimension keeps its two ghost planes,
 *              the other dimensions are periodic and stored without ghosts:
 *              3-D [nloc+2][Ty][Tx], 2-D [nloc+2][Tx], 1-D [nloc+2].
 *              Vector grids (E) hold 3 doubles per node (xyz, value-major as
 *              grid.c:413-500).
 *   global     the whole periodic domain without ghosts [Tz][Ty][Tx] (MG,
 *              spectral); with one rank it aliases the slab's true planes.
 */
#ifndef PINC_HIP_H
#define PINC_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define PINC_MAX_SPECIES 8
#define PINC_MAX_LEVELS 12

/* geometry of one rank's slab; dims ordered x,y,z; slab dim = nd-1 */
typedef struct {
	int nd;        /* 1..3 */
	int T[3];      /* global true size per dim (1 for unused dims) */
	int nloc;      /* true cells of this rank along the slab dimension */
	int off;       /* first true cell of this rank along the slab dim */
	int nranks;    /* slabs along the slab dimension */
	int literal;   /* main.c's double rho FROMHALO (literal loop): 1 = deposits on
	                  periodic ghost nodes of the non-slab dims count twice per
	                  ghost coordinate; 2 = only the weight a plain deposit
	                  misses for a second fold, (2^g - 1) per weight, doubled on
	                  slab ghost planes (the second fold adds them once more) */
} pinc_geom_t;

/* a population on the device (by value; pointers are device pointers) */
typedef struct {
	double *x[3];
	double *v[3];
	int nSpecies;
	int nd;
	long iStart[PINC_MAX_SPECIES + 1];
	long iStop[PINC_MAX_SPECIES];
} pinc_pop_t;

/* ------------------------------------------------------------ runtime -- */
const char *pinc_hip_error_string(void);
int pinc_hip_set_device(int dev);
int pinc_hip_device_count(int *n);
int pinc_hip_stream_create(void **stream);
/* Stream capture of a fixed launch sequence into a graph (MG V-cycle replay;
 * replaces the reference's per-call dispatch, no reference counterpart):
 * begin on a non-default stream, end -> instantiated executable, launch on a
 * stream, destroy. */
int pinc_hip_capture_begin(void *stream);
int pinc_hip_capture_end(void *stream, void **exec);
int pinc_hip_graph_launch(void *exec, void *stream);
int pinc_hip_graph_destroy(void *exec);
int pinc_hip_stream_destroy(void *stream);
int pinc_hip_stream_sync(void *stream);
int pinc_hip_device_sync(void);
int pinc_hip_malloc(void **ptr, unsigned long bytes);
int pinc_hip_free(void *ptr);
int pinc_hip_memset(void *ptr, int value, unsigned long bytes, void *stream);
int pinc_hip_h2d(void *dst, const void *src, unsigned long bytes, void *stream);
int pinc_hip_d2h(void *dst, const void *src, unsigned long bytes, void *stream);
int pinc_hip_d2d(void *dst, const void *src, unsigned long bytes, void *stream);
/* asynchronous device-to-host copy (dst: pinned memory from
 * pinc_hip_host_alloc), complete once an event recorded after it is
 * (pinc_hip_event_sync): the host keeps enqueueing work meanwhile (the
 * multigrid's per-cycle norm, pinc_mg.c) */
int pinc_hip_d2h_async(void *dst, const void *src, unsigned long bytes, void *stream);
int pinc_hip_host_alloc(void **ptr, unsigned long bytes);
int pinc_hip_host_free(void *ptr);
int pinc_hip_event_sync(void *ev);
/* events for per-phase device timing (replaces Timer, aux.c:48-85) */
int pinc_hip_event_create(void **ev);
int pinc_hip_event_destroy(void *ev);
int pinc_hip_event_record(void *ev, void *stream);
int pinc_hip_event_elapsed(float *ms, void *start, void *stop);
int pinc_hip_mem_info(unsigned long *freeBytes, unsigned long *totalBytes);

/* --------------------------------------------------------- particles -- */
/* puMove (pusher.c:86-119, as compiled: pos += vel) fused with the
 * neighbour classification of puExtractEmigrants3D/ND (pusher.c:782-910):
 * flags[i] = ne in 0..3^nd-1, center = stays.  chunkCount[b] = emigrants of
 * chunk b (PINC_CHUNK particles).  If doMove is 0 only classifies.
 * thr = [lower(nd), upper(nd), size-1 (nd)] as MpiInfo.thresholds.
 * wrapMask bit d (tiled layout only): a crossing in dimension d is applied in
 * place with the import's periodic shift and does not count as emigration;
 * 0 reproduces the reference exactly. */
#define PINC_CHUNK 2048
int pinc_hip_move_classify(pinc_pop_t pop, int s, int doMove, const double *thr,
                           unsigned char *flags, int *chunkCount, double maxVel,
                           int *errFlag, int wrapMask, void *stream);

/* Fused push of species s: optionally puAcc's kick
 * (kick=1: gather from Es as pinc_hip_accelerate, v += dv, KE partials of
 * blocks of PINC_CHUNK/2 particles in kePartial, *nBlocks of them), then
 * puMove's drift, the classification of pinc_hip_move_classify (flags,
 * chunkCount -- zeroed by the caller -- errFlag, wrapMask) and the CIC
 * deposit (puDistr3D1/ND1 weights) of every particle that stays into the
 * species accumulator rhoS (slab layout, not zeroed here).
 *   cursor == NULL: particle i stays at i; new positions go to xout (may be
 *     pop.x), velocities to vout (may be pop.v).
 *   cursor != NULL (tiled layout, sorted output): particle i goes to slot
 *     cursor[key(x_i)]++ (cursor = exclusive scan of the key counts of the
 *     current positions, pinc_hip_count_keys + pinc_hip_scan_keys), its
 *     moved state to xout/vout at that slot (must not alias pop), flags at
 *     that slot; chunkCount counts emigrants per destination chunk.
 *     Otherwise (cursor == NULL) the keys of the moved particles that stay
 *     are counted into cntNext if set (zeroed by the caller); a sorting
 *     push does not count. */
typedef struct {
	double *xout[3];
	double *vout[3];
	int kick;
	const double *Es;
	double *rhoS;
	const double *thr;
	unsigned char *flags;
	int *chunkCount;
	double maxVel;
	int *errFlag;
	int wrapMask;
	double *kePartial;
	int tileWidth;
	int *cursor;
	int *cntNext;
	unsigned long long *moved; /* if set: += particles that stay and changed cell */
	unsigned long long *spread; /* if set: += each block's input cell-box volume (cells spanned by its
	                             * items, periodic images nearest its first item) */
	unsigned long long *tstamp; /* if set: 8 phase timestamps per block (diagnostics) */
	unsigned long long *diag;   /* if set: [0] += items of a sorting push given a global slot one by
	                             * one (outside its LDS boxes; diagnostics) */
	/* immersed objects (fused collection, oCollectObjectCharge's test at
	 * object.c:489-494 on the moved position): if objInside is set, a
	 * particle that stays and whose cell's lower node has an object id > 0
	 * in objInside (padded local nodes, strides 1, objSy, objSz; objNodes
	 * nodes) is flagged PINC_NE_SINK instead of deposited, and counted in
	 * objCount[id - 1] */
	const unsigned char *objInside;
	long objSy, objSz, objNodes;
	int *objCount;
	int objLo[3], objHi[3];   /* bounding box (padded node coordinates, inclusive)
	                             of the nodes with an id: only cells there are looked up */
	unsigned long long *emigTotal; /* if set: += the particles flagged to leave (every flag but the
	                                  centre: emigrants, collected, outside the frame) */
	int flagsSparse;  /* 1: write only the flags that are not the centre (every other flag of the
	                     species' range must already be the centre: pinc_hip_extract puts the
	                     extracted particles' flags back to it); 0: write every live particle's flag */
} pinc_push_t;
int pinc_hip_push(pinc_pop_t pop, int s, pinc_geom_t g, const pinc_push_t *args, int *nBlocks, void *stream);
/* number of sort keys (cells incl. the wrap layer) of the tiled layout */
long pinc_hip_tile_keys(pinc_geom_t g, int tileWidth);
/* counts[key(x_i)] += 1 for particles iStart[s]+first .. iStop[s]-1 */
int pinc_hip_count_keys(pinc_pop_t pop, int s, long first, pinc_geom_t g, int tileWidth, int *counts, void *stream);
/* exclusive scan of nKeys counts (offsets[nKeys] = total); work holds
 * 2*ceil(nKeys/4096)+1 ints */
int pinc_hip_scan_keys(const int *counts, long nKeys, int *offsets, int *work, void *stream);
/* puBoris3D1KE (pusher.c:433-483; rotation parameters pusher.c:485-505) with
 * the reference's indexing defect corrected: per particle a half kick from
 * Es (E as rescaled for species s), v' = v + v x T, v += v' x S (addCross
 * order), KE partial of v^2, half kick.  T, S: host pointers to species s's
 * three components each.  3-D only. */
int pinc_hip_boris(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es, const double *T, const double *S,
                   double *kePartial, int *nBlocks, void *stream);
/* rho = the reference's per-species chain (gZero; gMul(1/q_s); add species
 * s; gMul(q_s); pusher.c:512-572) applied to per-species sums acc[s], over
 * n slab elements */
int pinc_hip_rho_combine(double *rho, const double *const *acc, const double *charge, int ns, long n,
                         void *stream);

/* Tiled layout (population:layout = tiled, not in the reference): counting
 * sort of species s by cell, cells grouped in tiles of tileWidth^nd, from
 * pop into out (same ranges); the caller swaps the two.  nKeysOut returns
 * the number of keys K (cells incl. the wrap layer); work must hold
 * 2*(K+1) + 2*ceil(K/4096) + 1 ints (workCap), else an error is returned
 * with nKeysOut set.  Order within a cell is arbitrary. */
int pinc_hip_sort_tiles(pinc_pop_t pop, pinc_pop_t out, int s, pinc_geom_t g, int tileWidth,
                        int *work, long workCap, long *nKeysOut, void *stream);
/* Cell ranges of the last sort: work + (K+1) holds, after pinc_hip_sort_tiles,
 * the exclusive end of each cell's particle range.  puDistr over those
 * ranges: one thread per cell sums its particles' weights in registers;
 * particles that left their cell since the sort, and particles at index
 * >= nCell (appended since), are deposited individually. */
int pinc_hip_deposit_cells(pinc_pop_t pop, int s, pinc_geom_t g, int tileWidth, const int *cellEnds,
                           long nCell, double *rhoSlab, void *stream);

/* Emigrant extraction with the reference's back-fill order (pusher.c:
 * 782-855): survivors fill holes from the tail, emigrants are listed in the
 * exact order the serial loop extracts them, then stably bucketed by
 * direction.  Work arrays: see DESIGN.md "Migration".  Outputs:
 *   buf   (6 doubles per emigrant, SoA blocks of cap entries: x,y,z,vx,vy,vz)
 *   bufNe direction of each buffered emigrant
 *   neCount[PINC_NE_CODES] emigrants per direction (species s), then the
 *         particles a fused push collected into objects (PINC_NE_SINK)
 * Returns the number of emigrants in *nEmig.  Compacts species s in place
 * (iStop[s] decreases by *nEmig on the host side). */
typedef struct {
	int *chunkOffset;   /* nChunks+1 */
	int *scanWork;      /* 2*ceil(nChunks/4096)+1 (multi-block scan of the chunk counts) */
	int *tail;          /* >= nEmig+1 */
	int *holes;         /* >= nEmig+1 */
	int *order;         /* >= nEmig   */
	int *blockHist;     /* >= 28*ceil(nEmig/1024)+28 */
	int *scratch;       /* >= 64 ints */
	double *buf;        /* 6*cap doubles */
	unsigned char *bufNe;
	long cap;
} pinc_extract_ws_t;
#define PINC_ERR_CAPACITY 77  /* *nEmig emigrants exceed ws.cap: grow and retry */
/* flag of a particle collected by an object in the fused push: extracted
 * like an emigrant, after every direction (neCount[PINC_NE_SINK]); neCount
 * has PINC_NE_CODES entries */
#define PINC_NE_SINK 27
#define PINC_NE_CODES 28
/* The flags of the extracted particles are set back to the centre, so that a
 * species' flags are all the centre again after its extraction. */
int pinc_hip_extract(pinc_pop_t pop, int s, unsigned char *flags, int *chunkCount,
                     int center, int nNeighbors, pinc_extract_ws_t ws, long *nEmig,
                     long *neCount, void *stream);

/* immersed objects (k_objects.hip; object.c, config C5).  inside: one byte
 * per node of the padded reference layout (strides 1, sy, sz; nNodes
 * nodes), the object id of interior nodes (0: none).  obj_flag writes
 * flags/chunk counts in pinc_hip_extract's format (flag 0 = remove, 13 =
 * keep) for oCollectObjectCharge (object.c:460-515) and adds the flagged
 * particles per object to objCount[id-1].  idx: device indices of the
 * surface nodes in a grid's slab storage.  obj_correct adds
 * sum_j M[j*n+i] (phiC - phiS[j]) to rho[idx[i]] (object.c:349-362). */
int pinc_hip_obj_flag(pinc_pop_t pop, int s, const unsigned char *inside, long sy, long sz, long nNodes,
                      unsigned char *flags, int *chunkCount, int *objCount, void *stream);
int pinc_hip_obj_gather(const double *grid, const long *idx, long n, double *out, void *stream);
int pinc_hip_obj_correct(const double *M, const double *phiS, long n, double phiC, const long *idx, double *rho,
                         void *stream);
int pinc_hip_obj_add(double *grid, const long *idx, long n, double v, void *stream);

/* multi-rank migration payload: records of 7 doubles (nd positions, nd
 * velocities, padding, direction) packed from buffer entries [first,
 * first+n), and appended to species s at index dst with the receiver's
 * shift (1-digit_d(ne))*T_d in every dimension (pusher.c:941-985) */
#define PINC_REC 7
int pinc_hip_pack(const double *buf, long cap, const unsigned char *bufNe, long first, long n,
                  int nd, double *out, void *stream);
int pinc_hip_import_rec(pinc_pop_t pop, int s, long dst, const double *rec, long n,
                        const int *shiftT, void *stream);

/* importParticles + shiftImmigrants (pusher.c:941-985): append n buffered
 * particles (buffer entries [first, first+n)) at index dst of species s,
 * shifting each position by -(digit_d(ne)-1)*T_d for the dims that wrap
 * locally (shiftMask bit d set). */
int pinc_hip_import(pinc_pop_t pop, int s, long dst, const double *buf, long cap,
                    const unsigned char *bufNe, long first, long n,
                    const int *shiftT, int shiftMask, void *stream);

/* CIC charge assignment puDistr3D1 / puDistrND1 (pusher.c:512-638) into the
 * slab grid; accumulates raw weights of species s (the caller applies the
 * reference's 1/q, q rescaling with pinc_hip_scale). */
int pinc_hip_deposit(pinc_pop_t pop, int s, pinc_geom_t g, double *rhoSlab, void *stream);

/* E as the reference holds it while species s is accelerated: its sequence
 * of in-place gMul(E, q/m) ... gMul(E, m/q) (pusher.c:192,212) gives
 * Es = E*pre; for t<s: Es = (Es*qm[t])*mq[t]; Es *= qm[s] (same rounding).
 * n doubles of the slab E grid; qm/mq are device arrays. */
int pinc_hip_field_chain(const double *E, double *Es, long n, const double *qm, const double *mq,
                         double pre, int s, void *stream);
/* Every species' Es of pinc_hip_field_chain in one pass over E (the same
 * running chain, bit-identical): species s at Es + s n, s < nSpecies. */
int pinc_hip_field_chain_all(const double *E, double *Es, long n, const double *qm, const double *mq, double pre,
                             int nSpecies, void *stream);

/* order 0 (nearest grid point, node (int)(x + 0.5)): puDistrND0
 * (pusher.c:640-668) adds one unit per particle of species s (the caller
 * applies the 1/q, q chain); puAccND0KE (pusher.c:310-353, puInterpND0
 * :1164-1180) v += Es at the node, KE partials as pinc_hip_accelerate */
int pinc_hip_deposit_ngp(pinc_pop_t pop, int s, pinc_geom_t g, double *rhoSlab, void *stream);
int pinc_hip_accelerate_ngp(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es, double *kePartial,
                            int *nBlocks, void *stream);
/* pVelAssertMax (population.c:342-365) over species s: a velocity component
 * above maxVel sets bit 0 of *errFlag */
int pinc_hip_vel_assert(pinc_pop_t pop, int s, double maxVel, int *errFlag, void *stream);
/* particles per workgroup of pinc_hip_push (a build constant) */
long pinc_hip_push_chunk(void);
/* xcd[c] = the XCD (block index mod 8) whose block processes push chunk c,
 * for a launch of nBlocks blocks (the push's chunk placement; trace
 * diagnostics) */
int pinc_hip_push_xcd_of_chunks(long nBlocks, int *xcd);

/* puAcc3D1KE / puAccND1KE (pusher.c:178-265) with puInterp3D1/ND1
 * (pusher.c:1089-1162), gathering from Es (pinc_hip_field_chain).
 * kePartial receives per-block partial sums of v.(v+dv) (at most
 * ceil((n+1)/2048) blocks); nBlocks returned. */
int pinc_hip_accelerate(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es,
                        double *kePartial, int *nBlocks, void *stream);

/* device-side initial conditions (pPosLattice population.c:172-240,
 * pPosPerturb 242-276, pVelZero/Maxwell): generates the lattice indices of
 * this rank, optional cosine perturbation, zero or Maxwellian velocities
 * from the counter RNG shared with the oracle.  Returns count in *n. */
int pinc_hip_init_species(pinc_pop_t pop, int s, pinc_geom_t g, long nGlobal, double latticeStep,
                          const int *subdomain, const int *nSubdomains, const int *offset,
                          const double *amp, const double *mode, int perturb,
                          int maxwell, double drift, double vth, unsigned long long seed,
                          long *n, void *stream);

/* -------------------------------------------------------------- grids -- */
int pinc_hip_zero(double *a, long n, void *stream);
int pinc_hip_scale(double *a, long n, double f, void *stream);
/* a = (a*f1)*f2 in one pass (two roundings, as two gMul calls) */
int pinc_hip_scale2(double *a, long n, double f1, double f2, void *stream);
/* gHaloOp(addSlice, rho, FROMHALO) along the slab dim for a self-periodic
 * slab (grid.c:340-406): plane 0 += into nloc, plane nloc+1 += into 1 */
int pinc_hip_fold_self(double *slab, pinc_geom_t g, void *stream);
/* a += b elementwise (gAddTo, grid.c:781-789) */
int pinc_hip_add(double *a, const double *b, long n, void *stream);
/* every slab node (incl. ghost planes) from the global periodic grid:
 * gHaloOp(setSlice, TOHALO) for a grid whose truth lives in the global
 * array (phi after the solve) */
int pinc_hip_slab_from_global(double *slab, const double *global, pinc_geom_t g, int nValues,
                              void *stream);
/* add a received plane into a slab plane */
int pinc_hip_add_plane(double *slab, pinc_geom_t g, int plane, const double *in, void *stream);
int pinc_hip_copy_plane(double *dst, const double *slab, pinc_geom_t g, int plane, int nValues, void *stream);
/* gFinDiff1st + TOHALO (grid.c:226-261, main.c:245-246):
 * E = 0.5*(phi[+d]-phi[-d]) on every slab plane incl. ghosts, from the
 * global periodic phi (ghost planes then equal the neighbours' values
 * bit for bit, so the TOHALO is implied). */
int pinc_hip_efield(const double *phiGlobal, pinc_geom_t g, double *Eslab, void *stream);
/* The same with E = h (phi_up - phi_dn): h = 0.5 is pinc_hip_efield, h = -0.5
 * its result followed by gMul(E, -1) (main.c:247) bit for bit, in one pass
 * (regular()'s step); other h are rejected. */
int pinc_hip_efield_scaled(const double *phi, pinc_geom_t g, double *E, double h, void *stream);
/* deterministic two-stage sums: *out = sum(a) ; sum(a*b) */
int pinc_hip_sum(const double *a, long n, double *partial, double *out, void *stream);
int pinc_hip_dot(const double *a, const double *b, long n, double *partial, double *out, void *stream);
/* *out = sum(a)/div  (the mean of gNeutralizeGrid, grid.c:746) */
int pinc_hip_sum_div(const double *a, long n, double div, double *partial, double *out, void *stream);
/* *out = (sum of the first n entries of partial) / div */
int pinc_hip_reduce(const double *partial, int n, double div, double *out, void *stream);

/* --------------------------------------------------------- multigrid -- */
/* One level of the global periodic grid. */
typedef struct { int nd; int T[3]; } pinc_lvl_t;
/* Red-black Gauss-Seidel colour pass (mgGS3D multigrid.c:683-767 when nd3,
 * mgGSND 553-621 otherwise) on true points of colour `pass`, reading the
 * other colour with the pending neutralisation shift *muPrev (exactly the
 * reference's stored value - mu), writing block partial sums of the
 * resulting logical grid into partial. nBlocks returned. */
int pinc_hip_gs_pass(double *phi, const double *rho, pinc_lvl_t L, int pass, int nd3,
                     const double *muPrev, double *partial, int *nBlocks, void *stream);
/* phi = (phi - muA) - muB on colour `pass`'s complement and phi - muB on
 * colour `pass` (materialise pending shifts after a smoothing sequence) */
/* Native mode (multigrid:native): one full red-black iteration of mgGS3D
 * without the per-colour neutralisation, phiIn -> phiOut (distinct buffers),
 * in one pass; bit-identical to two pinc_hip_gs_pass calls with muPrev NULL.
 * Needs a 3-D level with T[0], T[1], T[2] multiples of 16. */
int pinc_hip_gs_sweep(const double *phiIn, double *phiOut, const double *rho, pinc_lvl_t L,
                      void *stream);
/* Native mode: two full red-black iterations phiIn -> phiOut in one pass
 * (z-march four stages deep); bit-identical to two pinc_hip_gs_sweep calls.
 * Needs T[0] % 32, T[1] % 8 and T[2] % 16 == 0. */
int pinc_hip_gs_sweep2x(const double *phiIn, double *phiOut, const double *rho, pinc_lvl_t L,
                        void *stream);
/* Native mode: the whole V-cycle below (and including) a coarse level in one
 * 1024-thread workgroup, grids in LDS (at most 5500 points over all levels,
 * 1-D to 3-D, each level half the previous in every dimension).  levels[0]
 * is the top coarse level: its rho is read from `rho`, its correction starts
 * at zero and is written to `phi`; rho of the levels below is the restricted
 * residual times 4.  hw3d / gs3d select mgHalfRestrict3D / mgGS3D's forms
 * (3-D only), else the ND forms. */
/* Native mode, one rank, a 2-D level 0 of T0 x T1 <= 16384 points (T0 a
 * power of two, T1 even, T0 T1 a multiple of 2048; mgGSND form, the ND
 * restriction), levels 1.. within k_mg_coarse's LDS budget: whole V-cycles
 * of levels[0..nLevels) from phi (initial guess, in/out) with rho, in one
 * workgroup, until the RMS residual is <= tol or maxCycles ran; res (T0 T1
 * doubles) is scratch.  out[0] = cycles, out[1] = the last RMS residual,
 * out[2 + c] = the residual after cycle c (c < 60).  coarseBasis NULL: the
 * V-cycle of the per-level launches (k_mg_coarse for levels 1..);
 * otherwise the two-grid cycle of multigrid:spectralCoarse with level 1
 * (square, n = 16..64 in 16s) solved exactly: coarseBasis holds the real
 * orthonormal Fourier basis Q (n x n, row-major, Q[j][k]) and then the n
 * eigenvalues 2 - 2 cos(2 pi f_k / n) of its columns. */
int pinc_hip_mg_solve_small(double *phi, const double *rho, double *res, int nLevels, const pinc_lvl_t *levels,
                            int nPre, int nPost, int nCoarse, int maxCycles, double tol, const double *coarseBasis,
                            double *out, void *stream);
int pinc_hip_mg_coarse(const double *rho, double *phi, int nLevels, const pinc_lvl_t *levels, int nPre,
                       int nPost, int nCoarse, int hw3d, int gs3d, void *stream);
/* Sharded level 0 of the native multigrid (several ranks, 3-D): this rank's
 * z-slab extended by halo planes, Lx = T0 x T1 x (nloc + 2 hz), x/y periodic,
 * z neighbours read directly.
 *   residual_slab        residual on planes [zlo, zhi) of the extended slab
 *   residual_sumsq_slab  block partials of its square (RMS norm)
 *   restrict_slab        this rank's level-1 planes (Lc: T0/2 x T1/2 x nloc/2)
 *                        from the slab's residual starting at plane zf0,
 *                        times 4 (coarse h^2 factor)
 *   prolong_add_slab     every slab plane += the global level-1 correction
 *                        (Lc global); slab plane zl is global plane z0 + zl
 *                        (mod Tz)
 *   prolong_add_own      the owned planes [hz, hz + nloc) += the correction
 *                        of this rank's own level-1 planes, held in phiCx
 *                        with one halo plane on each side (Lcx: T0/2 x T1/2
 *                        x (nloc/2 + 2)); level 1 decomposed as level 0 */
int pinc_hip_residual_slab(double *res, const double *phi, const double *rho, pinc_lvl_t Lx, int zlo, int zhi,
                           void *stream);
int pinc_hip_residual_sumsq_slab(const double *phi, const double *rho, pinc_lvl_t Lx, int zlo, int zhi,
                                 double *partial, int *nBlocks, void *stream);
int pinc_hip_restrict_slab(const double *fineX, pinc_lvl_t Lx, int zf0, double *coarse, pinc_lvl_t Lc, int nd3,
                           void *stream);
int pinc_hip_prolong_add_slab(double *phiX, pinc_lvl_t Lx, int z0, int Tz, const double *phiC, pinc_lvl_t Lc,
                              void *stream);
int pinc_hip_prolong_add_own(double *phiX, pinc_lvl_t Lx, int hz, int nloc, const double *phiCx, pinc_lvl_t Lcx,
                             void *stream);
int pinc_hip_gs_materialize(double *phi, pinc_lvl_t L, int lastPass, const double *muA,
                            const double *muB, void *stream);
/* phi -= *mu over all points */
int pinc_hip_sub_dev(double *a, long n, const double *mu, void *stream);
/* multigrid:extrapolate (native mode, an extension): phi <- 2 phi - prev and
 * prev <- old phi over n values, the initial guess of the next solve from the
 * last two solutions (mgSolveRaw, multigrid.c:1688-1724, warm-starts from the
 * last one) */
int pinc_hip_extrapolate(double *phi, double *prev, long n, void *stream);
/* out = a x + b y over n values (out may alias x or y) */
int pinc_hip_lincomb(double *out, const double *x, double a, const double *y, double b, long n, void *stream);
/* mgResidual (multigrid.c:1385-1403): res = lap(phi) + rho */
int pinc_hip_residual(double *res, const double *phi, const double *rho, pinc_lvl_t L,
                      void *stream);
/* residual sum of squares only (mgSumTrueSquared, multigrid.c:1471-1481) */
int pinc_hip_residual_sumsq(const double *phi, const double *rho, pinc_lvl_t L,
                            double *partial, int *nBlocks, void *stream);
/* mgHalfRestrict3D / ND (multigrid.c:844-1022) */
int pinc_hip_restrict(const double *fine, double *coarse, pinc_lvl_t Lc, int nd3, void *stream);
/* mgBilinProl3D/ND + gAddTo (multigrid.c:1024-1238, 1535): phi_f += P(phi_c) */
int pinc_hip_prolong_add(double *phiFine, const double *phiCoarse, pinc_lvl_t Lf, void *stream);
/* 3-D forms of the level transfers, one thread per coarse cell (bit-identical
 * to the point kernels above): coarse = scale * restrict(residual(phi, rho))
 * (mgResidual + mgHalfRestrict3D / ND without writing the fine residual;
 * scale 4 in native mode); phi_f += P(phi_c) for the coarse level Lc (phi_f
 * 16-byte aligned) */
int pinc_hip_resid_restrict(const double *phi, const double *rho, double *coarse, pinc_lvl_t Lc, int hw3d,
                            double scale, void *stream);
int pinc_hip_prolong_add3(double *phiFine, const double *phiCoarse, pinc_lvl_t Lc, void *stream);

/* ---------------------------------------------------------- spectral -- */
/* Spectral Poisson solve on rocFFT, replacing sAlloc/sSolve/sFree
 * (spectral.c:14-52, 92-115).  T is the global true size (x fastest, x
 * even).  pinc_hip_fft_poisson reads the global rho [Tz][Ty][Tx] (left
 * unchanged) and writes the global phi: r2c, DC := 0, multiply by
 * (N/(2 pi n))^2/N in 1-D (spectral.c:29-37) or 1/|k|^2/N in 2-D/3-D, c2r. */
typedef struct pinc_fft_s pinc_fft_t;
int pinc_hip_fft_create(pinc_fft_t **plan, int nd, const int *T, void *stream);
int pinc_hip_fft_poisson(pinc_fft_t *plan, const double *rhoGlobal, double *phiGlobal, void *stream);
void pinc_hip_fft_destroy(pinc_fft_t *plan);
/* symbol of the plan's k-space factor: 0 the spectral solver's (above), 1
 * the multigrid's 7-point (5-, 3-point) discrete Laplacian,
 * 1/sum_d (2 - 2 cos(2 pi n_d/N_d))/N: the exact discrete solution the
 * multigrid converges to (objects:secondGuess = spectral) */
int pinc_hip_fft_set_symbol(pinc_fft_t *plan, int discrete);

/* Slab-distributed 3-D spectral solve (several ranks,
 * z-slabs of nloc planes, Ty divisible by the rank count): the same operator
 * as pinc_hip_fft_poisson without gathering rho.
 *   forward   rho slab (nloc planes, x fastest) -> batched 2-D r2c -> the
 *             send buffer S, blocks [q][zl][yl][kx] (block q: ky rows
 *             [q Ty/P, (q+1) Ty/P))
 *   (host)    block q of S to rank q into block r of B on rank q
 *   kspace    B = [z][yl][kx]: c2c along z, the k-space factor, inverse c2c
 *   (host)    block q of B (z rows of slab q) to rank q into block r of S
 *   backward  S -> unpack -> batched 2-D c2r -> phi slab (nloc planes)
 * buffers: S and B device pointers, bytes per block (P blocks each). */
typedef struct pinc_fft_slab_s pinc_fft_slab_t;
int pinc_hip_fft_slab_create(pinc_fft_slab_t **plan, const int *T, int nloc, int nranks, int rank, void *stream);
int pinc_hip_fft_slab_buffers(pinc_fft_slab_t *plan, void **S, void **B, long *blockBytes);
/* the slab plan's symbol, as pinc_hip_fft_set_symbol (1: the multigrid's
 * 7-point Laplacian; the sharded multigrid's spectral second guess) */
int pinc_hip_fft_slab_set_symbol(pinc_fft_slab_t *plan, int discrete);
int pinc_hip_fft_slab_forward(pinc_fft_slab_t *plan, const double *rhoSlab, void *stream);
int pinc_hip_fft_slab_kspace(pinc_fft_slab_t *plan, void *stream);
int pinc_hip_fft_slab_backward(pinc_fft_slab_t *plan, double *phiSlab, void *stream);
void pinc_hip_fft_slab_destroy(pinc_fft_slab_t *plan);

/* ------------------------------------------------------------ comm -- */
/* RCCL communicator over xGMI (one process per GPU).  id is the 128-byte
 * ncclUniqueId produced by pinc_hip_comm_unique_id on rank 0 and
 * distributed by the launcher. */
#define PINC_COMM_ID_BYTES 128
int pinc_hip_comm_unique_id(unsigned char *id);
int pinc_hip_comm_init(void **comm, const unsigned char *id, int nranks, int rank);
int pinc_hip_comm_destroy(void *comm);
/* label of the next RCCL call for the watchdog's message (pinc_hip_comm_init
 * starts a watchdog thread: a call that has not completed after
 * PINC_COMM_TIMEOUT seconds, default 300, aborts the communicator and ends
 * the process with status 3) */
int pinc_hip_comm_note(const char *what);
int pinc_hip_comm_sendrecv(void *comm, const void *sendbuf, long sendBytes, int peerSend,
                           void *recvbuf, long recvBytes, int peerRecv, void *stream);
/* grouped point-to-point exchange: op i sends sendBytes[i] to sendPeer[i]
 * and receives recvBytes[i] from recvPeer[i].  Transfers between one pair of
 * ranks match in op order, so with two slabs (up == down) pair each send
 * with the receive from the opposite direction. */
int pinc_hip_comm_exchange(void *comm, int nOps, const int *sendPeer, void *const *sendbuf,
                           const long *sendBytes, const int *recvPeer, void *const *recvbuf,
                           const long *recvBytes, void *stream);
int pinc_hip_comm_allgather(void *comm, const double *send, double *recv, long count, void *stream);
int pinc_hip_comm_allreduce_sum(void *comm, const double *send, double *recv, long count, void *stream);
/* test hook: occupy the stream for `seconds` (at most 30) of wall time with a
 * one-lane kernel that ends by itself (tests/test_gpu_rccl_watchdog.py holds
 * an RCCL call behind it) */
int pinc_hip_test_spin(double seconds, void *stream);

#ifdef __cplusplus
}
#endif
#endif
