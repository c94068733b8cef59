/*
 * kle.h -- C ABI of libkle.so, the MI355X-native KLE assembly + Krylov library.
 *
 * This is the drop-in boundary.  It replaces, for Pynama's hot path, the
 * petsc4py objects the reference creates and the Python element loops that
 * fill them (paths are under the reference's src/):
 *
 *   PETSc Mat (AIJ)  createAIJ/setValues/assemble/mult/diagonalScale
 *                      matrices/mat_fs.py:102-106,115-120,175-186,245-267
 *   PETSc Vec          createMPI/setValues/axpy/scale/dot/norm/...
 *                      matrices/mat_fs.py:228-236, cases/base_problem.py:129-154
 *   PETSc KSP/PC       KspSolver.createSolver / KleSolver.solve
 *                      solver/kle_solver.py:33-41,54-64
 *   MatFS.build element loops (buildFS, buildOperators)
 *                      matrices/mat_fs.py:131-201  -> kle_assemble_kle()
 *   DMPlex box mesh + FEM section numbering
 *                      domain/dmplex.py:31-49,193-196,382-388 -> kle_mesh_*
 *
 * Conventions (PETSc-like):
 *   - every function returns int: 0 = success, a KLE_ERR_* code otherwise;
 *     kle_last_error() returns a thread-local message for the last failure.
 *   - handles are opaque; plain pointers/sizes only, no torch types.
 *   - all device work is ordered on the context's HIP stream.
 *   - one process per GPU; ranks partition the mesh into slabs along the
 *     slowest lattice axis (z in 3-D, y in 2-D).  Collectives (halo exchange,
 *     Krylov dot products) go over RCCL inside the library.
 *   - handles are not thread-safe (same as PETSc objects).
 */
#ifndef KLE_H
#define KLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    KLE_OK = 0,
    KLE_ERR_ARG = 62,        /* PETSC_ERR_ARG_WRONG          */
    KLE_ERR_SIZ = 60,        /* PETSC_ERR_ARG_SIZ            */
    KLE_ERR_OUTOFRANGE = 63, /* PETSC_ERR_ARG_OUTOFRANGE     */
    KLE_ERR_MEM = 55,        /* PETSC_ERR_MEM                */
    KLE_ERR_SUP = 56,        /* PETSC_ERR_SUP (not supported) */
    KLE_ERR_STATE = 73,      /* PETSC_ERR_ARG_WRONGSTATE     */
    KLE_ERR_DEVICE = 76,     /* HIP runtime failure          */
    KLE_ERR_COMM = 98,       /* RCCL failure                 */
    KLE_ERR_NEWNZ = 77       /* insertion outside the preallocated pattern */
};

/* KSP converged reasons (same numeric values as PETSc's KSPConvergedReason). */
enum {
    KLE_CONVERGED_RTOL = 2,
    KLE_CONVERGED_ATOL = 3,
    KLE_CONVERGED_ITS = 4,
    KLE_DIVERGED_ITS = -3,
    KLE_DIVERGED_DTOL = -4,
    KLE_DIVERGED_BREAKDOWN = -5,
    KLE_DIVERGED_NANORINF = -9,
    KLE_CONVERGED_ITERATING = 0
};

typedef struct kle_ctx kle_ctx;
typedef struct kle_mesh kle_mesh;
typedef struct kle_vec kle_vec;
typedef struct kle_mat kle_mat;
typedef struct kle_ksp kle_ksp;

const char *kle_last_error(void);
/* Performance knobs for in-process A/B measurements (tools/cg_ab.py); every
 * value gives bitwise the same results, except the symmetric-storage keys
 * (the same product to rounding).  Keys: "spmv_waves" (0 auto, 4, 8:
 * rows per SpMV workgroup of 3x3 chunked matrices), "spmv_x_lds" (1 default:
 * structured 3x3 rows at 8 waves stage x in LDS; 0 off), "spmv_xcd_chunk"
 * (row blocks per XCD run, 0 round-robin; default 16), "spmv_dyn_lds" (unused
 * LDS bytes per SpMV workgroup while side-stream work runs, -1 auto),
 * "spmv_dict" (1 default: unstructured 3x3 rows at 8 waves read x through
 * per-group column dictionaries; 0 off), "spmv_dict_min_rows" (node rows from
 * which matrices get dictionaries at creation; default 64000), "upd_preload"
 * (1 default: CG update kernels load their first element and the stage inputs
 * before the prologue; 0 off), "upd_nt" (single-reduction CG update: every
 * vector but u loaded and stored nontemporal, so u stays in the Infinity
 * Cache for the SpMV; 0 off, 1 on, 2 auto = from 2M local entries), "spmv_sym" (1 default: matrices holding
 * symmetric storage run the symmetric SpMV; 0 the full storage),
 * "spmv_sym_min_rows" (node rows per rank from which kle_assemble_kle gives
 * K symmetric storage; default 40000), "spmv_sym_tz" (read when the storage
 * is built: 0 auto = 8 x 4 x 4-row tiles where two 8-wave workgroups fit a
 * CU, 2 = 8 x 8 x 2, 4 = 8 x 4 x 4), "spmv_sym_det" (1
 * default: the transposed adds as exact fixed-point sums, y bitwise
 * reproducible; 0 fp64 LDS atomics, reproducible to rounding),
 * "ksp_refine" (correction solves of new KSPs, kle_ksp_set_corrections:
 * default 2, 0 PETSc's plain stop -- KLE_KSP_REFINE),
 * "spmv_sym_waves" (0 auto, 8 or 16 waves per workgroup), "spmv_gsym_rows"
 * (read when the storage of an
 * unstructured K is built: rows per group, 64 default, 128, 32, 16 or 8),
 * "spmv_gsym_waves" (read at build: 0 auto = 16 for 64-row groups, else 8;
 * 8 or 16), "spmv_gsym_split" (read at build: the largest dictionary of the
 * first of its two launches; 0 auto), "spmv_sym_brick" (read at build:
 * the box K of one rank on bricks -- one 16-wave workgroup per CU, the
 * brick region's x and exact sums in LDS for the whole value stream; 1
 * default, 0 the 128-row tiles), "spmv_brick_max" (read at
 * build: at most this many bricks, 0 planned), "spmv_brick_rounds" (read at
 * build: at most this many bricks per CU, default 1), "spmv_brick_split" (read
 * at build: force nbx + 100 nby + 10000 nbz bricks, 0 planned),
 * "spmv_brick_pair" (read at build: rows in units of two whose last
 * partial 64-block passes share one item; 1 default), "spmv_brick_singles"
 * (read at build: rows of one stored block -- the Dirichlet rows and the
 * free rows at the far corner of their box -- formed by the gather instead
 * of as items of the bricks; 1 default), "spmv_gather_wps" (the run-mask
 * gather's waves per 64-row slice: 1, 2, 4; 0 default, by the runs per
 * slice), "spmv_gsym_brick" (read at build: graph K on graph bricks, whole
 * rounds per CU; 1 default), "ipc_sentinel" (IPC transport debug mode:
 * consumed mailbox slots overwritten with NaN before the ack; 0 default),
 * "ksp_corr_fault" (test hook: correction solves that end in NaN; 0),
 * "upd_unroll" (CG update kernel: 1 default or 2), "ksp_pipe_gather" (box
 * bricks: the pipelined CG's update gathers the split product itself; 1
 * default, 0 a separate gather launch), "ksp_sr_gather" (the same for the
 * single-reduction CG at one rank, the bricks forming (A u, u): 1 default
 * from 2^17 node rows, 2 always, 0 never),
 * "spmv_sym_tile64" (read at build: 8 x 2 x 4-row tiles -- 0 auto, below
 * "spmv_sym_tile64_max" (640) 128-row tiles; 1 wherever two workgroups fit
 * a CU; 2 never), "spmv_sym_ovl_b" (N > 1, box symmetric SpMV with halo
 * overlap: the percentage of the interior tiles run beside the reverse halo,
 * the rest beside the forward halo; default 50), "spmv_sym_early" (box tile kernel loads its first items before
 * x is in LDS; 0 default), "spmv_sym_align" (read at build: partial slots
 * aligned to 128-B lines; 0 default), "spmv_sym_stpol"
 * (box kernel's partial stores: 0 plain default, 1 nontemporal, 2 sc1, 3 sc0
 * sc1), "spmv_gsym_stpol" (the same for the graph kernel; default 2).
 * Every value gives correct results (the
 * timing probes of the symmetric SpMV exist only in the tools/ probe build,
 * `make -C pynama_amd/csrc probe`). */
int kle_set_tuning(const char *key, int value);
int kle_get_tuning(const char *key, int *value);
int kle_version(void);

/* ---------------------------------------------------------------- context */
/* 128-byte RCCL unique id, produced on rank 0 and broadcast by the caller. */
int kle_get_unique_id(unsigned char out[128]);
/* device: HIP ordinal; nranks==1 needs no unique id (pass NULL). */
int kle_ctx_create(int device, int rank, int nranks, const unsigned char *unique_id,
                   kle_ctx **out);
/* Host-staged transport (testing / debugging): the same distributed code
 * paths with the collectives delegated to caller callbacks on host buffers
 * (e.g. gloo), so several ranks can share one GPU.  Production runs use RCCL.
 *   allreduce: in-place sum of n doubles over all ranks.
 *   halo: send n_send_lo doubles to lo_rank and n_send_hi to hi_rank, receive
 *         n_recv_lo from lo_rank and n_recv_hi from hi_rank (ranks < 0: none).
 *   exchange: general halo of graph-partitioned meshes: for peer k send
 *         send_cnt[k] doubles (packed back to back in `send`, peer order) and
 *         receive recv_cnt[k] (packed in `recv`); may be NULL when no mesh
 *         with a graph partition is used. */
typedef struct {
    int (*allreduce)(double *buf, int n, void *user);
    int (*halo)(const double *send_lo, int64_t n_send_lo, int lo_rank, const double *send_hi,
                int64_t n_send_hi, int hi_rank, double *recv_lo, int64_t n_recv_lo,
                double *recv_hi, int64_t n_recv_hi, void *user);
    void *user;
    int (*exchange)(int npeers, const int *peers, const double *send, const int64_t *send_cnt,
                    double *recv, const int64_t *recv_cnt, void *user);
} kle_host_comm;
int kle_ctx_create_host_comm(int device, int rank, int nranks, const kle_host_comm *comm,
                             kle_ctx **out);
/* Device-to-device transport for a host-comm context (KLE_TRANSPORT=ipc;
 * collective): every rank exports one mailbox (hipIpcGetMemHandle, handles
 * exchanged over the host callbacks) and maps the others'; the slab halos,
 * the symmetric SpMV's reverse halo and the allreduces then run as
 * hipMemcpyAsync copies into the peers' mailboxes with stream wait/write-value
 * signals (no host staging, no RCCL kernels on the SpMV's CUs; the allreduce
 * sums the ranks' slots in rank order, the same bits on every rank).  Graph-
 * partition halos keep the host path.  KLE_ERR_COMM when any rank cannot
 * export or map (then no rank switches). */
int kle_ctx_enable_ipc(kle_ctx *ctx);
int kle_ctx_destroy(kle_ctx *ctx);
int kle_ctx_synchronize(kle_ctx *ctx);
int kle_ctx_barrier(kle_ctx *ctx); /* device-side RCCL barrier + stream sync */
/* Diagnostics (no reference counterpart): the HIP ordinal, its PCI bus id
 * (may be NULL) and the transport: 0 single rank, 1 RCCL, 2 host-staged,
 * 3 IPC mailboxes (kle_ctx_enable_ipc). */
int kle_ctx_get_device(kle_ctx *ctx, int *device, char *pci_bus_id, int len, int *transport);
/* What the RCCL communicator itself reports (ncclCommCount /
 * ncclCommUserRank; the MPI communicator of DMPlex.distribute, dmplex.py:21,
 * and of KSPSolve's reductions, kle_solver.py:35): *count = 0, *rank = -1
 * when the context has no RCCL communicator (one rank, host or IPC transport). */
int kle_ctx_get_comm_info(kle_ctx *ctx, int *count, int *rank);
/* Diagnostic, host only (no device, no reference counterpart): the brick
 * plan of the symmetric SpMV for an Lx x Ly x Lz box lattice of p-node
 * elements (dirichlet: boundary rows the diagonal alone) on ncu CUs, at
 * most `rounds` bricks per CU (split: forced counts nbx + 100 nby + 10000 nbz, 0
 * planned).  info[5]: bricks, bricks along x / y / z, LDS bytes; stats[6]:
 * largest brick's bytes over the mean, region entries per row, stored blocks,
 * modelled microseconds, 64-lane items streamed, share of their lanes that
 * carry a block. */
int kle_brick_plan_box(int Lx, int Ly, int Lz, int p, int dirichlet, int ncu, int rounds, int split, int *info,
                       double *stats);
/* Per-kernel HIP-event timing of the hot kernels (SpMV, CG updates). */
int kle_ctx_set_profiling(kle_ctx *ctx, int on);
/* Time only the launches tagged `name` ("spmv", "dot", "cg_update", "reduce",
 * "halo", "allreduce"); NULL or "" times all of them. */
int kle_ctx_set_profiling_filter(kle_ctx *ctx, const char *name);
/* Time only one launch in `every` of the profiled tags (1 = all): keeps the
 * event overhead out of a timed loop while still sampling it live. */
int kle_ctx_set_profiling_sample(kle_ctx *c, int every);
/* name: "spmv" | "cg_update" | "p_update" | "reduce" | "halo" | "allreduce" */
int kle_ctx_get_kernel_stats(kle_ctx *ctx, const char *name, int64_t *count, double *total_ms);
int kle_ctx_reset_kernel_stats(kle_ctx *ctx);

/* ------------------------------------------------------------------- mesh */
/* Structured box mesh (replaces BoxDom.create + DMPlexDom.setFemIndexing,
 * dmplex.py:31-49,382-388).  Host-only: usable without a GPU.  Node ids are
 * lattice-lexicographic (x fastest); cells x-fastest; element-local nodes in
 * tensor order. */
int kle_mesh_create_box(int dim, const int64_t nelem[3], const double lower[3],
                        const double upper[3], int ngl, int rank, int nranks, kle_mesh **out);
int kle_mesh_destroy(kle_mesh *m);
/* Unstructured quad (2-D) / hex (3-D) mesh (replaces GmshDom.create +
 * DMPlexDistribute + setFemIndexing, dmplex.py:18-49,390-395; entity
 * orientation rules indices.py:70-96).  vxyz: [nverts][3]; cells:
 * [ncells][2^dim] vertex indices in Gmsh order (quad counter-clockwise, hex
 * bottom 0-3 then 4-7 above them), cell ids = row order (the ADD order);
 * facets: [nfacets][2^(dim-1)] boundary faces with their Face Sets value
 * (tag t >= 1 -> face bit t-1, the reference's name order: dmplex.py:27-30,
 * 175-178).  Cells are partitioned by kle_set_partitioner's method; node ids
 * are global, owned ranges contiguous per rank (see kle_umesh.cpp).  Fails
 * with KLE_ERR_ARG for inverted cells, ranks without nodes, or slabs too thin
 * for the two-neighbour halo. */
int kle_mesh_create_unstructured(int dim, int ngl, int64_t nverts, const double *vxyz, int64_t ncells,
                                 const int64_t *cells, int64_t nfacets, const int64_t *facets,
                                 const int *facet_tags, int rank, int nranks, kle_mesh **out);
/* Gmsh MSH 4.1 ASCII file (GmshDom.create -> DMPlexCreateFromFile). */
int kle_mesh_create_gmsh(const char *path, int ngl, int rank, int nranks, kle_mesh **out);
/* Partitioner of the unstructured meshes created afterwards (the role of
 * DMPlexDistribute's Chaco partitioner, dmplex.py:21): 0 (default) inertial
 * recursive bisection of the cells -- general partitions, any number of
 * neighbours per rank, index-list halos; 1 slabs along the longest axis
 * (two-neighbour halo in contiguous ranges). */
int kle_set_partitioner(int method);
int kle_get_partitioner(void);
/* Halo of a rank: npeers neighbours, per peer its rank, the ghost nodes
 * received and the owned nodes sent; send_list (optional, sum of send_nodes
 * entries) holds the owned-local node indices sent, peer by peer. */
int kle_mesh_get_peers(const kle_mesh *m, int *npeers, int *ranks, int64_t *recv_nodes, int64_t *send_nodes,
                       int64_t *send_list);
/* Global node id of every ext (owned + ghost) node, in ext order. */
int kle_mesh_get_ext_gids(const kle_mesh *m, int64_t *gids);
/* Global cell ids of the local (owned + ghost) elements, ascending. */
int kle_mesh_get_elements(const kle_mesh *m, int64_t *ids);

typedef struct {
    int dim, ngl, rank, nranks;
    int64_t nelem[3];
    int64_t lattice[3];     /* nodes per axis                                */
    int64_t n_nodes;        /* global                                        */
    int64_t n_elems;        /* global                                        */
    int64_t node_begin;     /* owned node range [node_begin, node_end)       */
    int64_t node_end;
    int64_t ext_begin;      /* owned + ghost node range [ext_begin, ext_end) */
    int64_t ext_end;
    int64_t elem_begin;     /* local (owned + ghost) element range           */
    int64_t elem_end;
    int kind;               /* 0 structured box, 1 unstructured              */
    int axis;               /* partition axis                                */
} kle_mesh_info;

int kle_mesh_get_info(const kle_mesh *m, kle_mesh_info *info);
/* element->global node ids for local elements, tensor order [elem][ngl^dim]. */
int kle_mesh_get_conn(const kle_mesh *m, int64_t *conn);
/* cell corners in DMPlex closure order [elem][2^dim][dim] (dmplex.py:93-100). */
int kle_mesh_get_corners(const kle_mesh *m, double *xyz);
/* coordinates of the owned nodes [node][dim] (computeFullCoordinates). */
int kle_mesh_get_coords(const kle_mesh *m, double *xyz);
/* Boundary nodes of named faces: face bit f follows the reference's naming
 * (dmplex.py:27-30): 3-D 0 back(z-) 1 front(z+) 2 down(y-) 3 up(y+) 4 right(x+)
 * 5 left(x-); 2-D 0 down 1 right 2 up 3 left.  Fills the owned boundary
 * nodes (sorted) and returns their count in *n (pass nodes=NULL to count). */
int kle_mesh_face_nodes(const kle_mesh *m, unsigned face_mask, int64_t *nodes, int64_t *n);
/* Dirichlet (free-slip) node set: faces by mask, or explicit global ids. */
int kle_mesh_set_dirichlet_faces(kle_mesh *m, unsigned face_mask);
int kle_mesh_set_dirichlet_nodes(kle_mesh *m, const int64_t *nodes, int64_t n);
/* No-slip walls (BoundaryConditions.getNoSlipTangDofs / getNoSlipNormalDofs,
 * boundary_conditions.py:214-241): global velocity DoF ids; a DoF in both
 * lists is normal (mat_ns.py:60-62).  Their nodes become the fixed nodes. */
int kle_mesh_set_noslip_dofs(kle_mesh *m, const int64_t *tang, int64_t nt, const int64_t *normal, int64_t nn);
/* Same, from the no-slip faces (face bits as kle_mesh_set_dirichlet_faces) in
 * the order the configuration lists them (that order decides corner DoFs). */
int kle_mesh_set_noslip_faces(kle_mesh *m, const int *faces, int nfaces);
/* Symbolic node-block pattern (host).  which: 0 K, 1 Krhs, 2 Rw, 3 operators
 * (Curl/SrT/DivSrT: every node x every node sharing a cell).
 * row_ptr[n_owned+1] (block offsets, unpadded) and col[] (global node ids). */
int kle_mesh_pattern_size(const kle_mesh *m, int which, int64_t *nblocks);
int kle_mesh_pattern(const kle_mesh *m, int which, int64_t *row_ptr, int64_t *cols);
/* Halo plan of this rank (node counts): ghosts received from below/above,
 * owned nodes sent to the lower/upper neighbour, neighbour ranks (-1: none). */
int kle_mesh_halo(const kle_mesh *m, int64_t *lo_count, int64_t *hi_count, int64_t *send_lo,
                  int64_t *send_hi, int *lo_rank, int *hi_rank);

/* -------------------------------------------------------------------- vec */
/* Mesh vector with bs components per node, ghosted over the ext range. */
int kle_vec_create_mesh(kle_ctx *ctx, const kle_mesh *m, int bs, kle_vec **out);
/* Plain distributed vector (no ghosts). */
int kle_vec_create(kle_ctx *ctx, int64_t n_local, int64_t n_global, kle_vec **out);
int kle_vec_duplicate(const kle_vec *v, kle_vec **out);
int kle_vec_destroy(kle_vec *v);
int kle_vec_get_sizes(const kle_vec *v, int64_t *n_local, int64_t *n_global);
int kle_vec_get_ownership_range(const kle_vec *v, int64_t *lo, int64_t *hi);
int kle_vec_set(kle_vec *v, double alpha);
int kle_vec_copy(const kle_vec *x, kle_vec *y);                 /* y = x          */
int kle_vec_axpy(kle_vec *y, double alpha, const kle_vec *x);   /* y += a x       */
int kle_vec_aypx(kle_vec *y, double beta, const kle_vec *x);    /* y = x + b y    */
int kle_vec_waxpy(kle_vec *w, double alpha, const kle_vec *x, const kle_vec *y); /* w = a x + y */
int kle_vec_scale(kle_vec *v, double alpha);
int kle_vec_pointwise_mult(kle_vec *w, const kle_vec *x, const kle_vec *y);
/* out[node] = v v^T of the dim-vector at each node, components xx,xy,yy
 * (2-D) or xx,xy,yy,yz,zz,zx (3-D): BaseProblem.computeVtensV
 * (base_problem.py:138-154). */
int kle_vec_tensor_square(const kle_vec *v, int dim, kle_vec *out);
int kle_vec_reciprocal(kle_vec *v);
int kle_vec_dot(const kle_vec *x, const kle_vec *y, double *out);
int kle_vec_norm2(const kle_vec *x, double *out);
/* Host <-> device.  Indices are GLOBAL; only owned entries may be set.
 * addv: 0 INSERT_VALUES, 1 ADD_VALUES (applied in index order). */
int kle_vec_set_values(kle_vec *v, int64_t n, const int64_t *idx, const double *vals, int addv);
int kle_vec_get_values(const kle_vec *v, int64_t n, const int64_t *idx, double *vals);
int kle_vec_get_array(const kle_vec *v, double *host_local);     /* owned part */
int kle_vec_set_array(kle_vec *v, const double *host_local);
/* petsc4py getArray()/restoreArray pair: kle_vec_get_array copies the owned
 * part out, kle_vec_restore_array writes a (modified) host copy back. */
int kle_vec_restore_array(kle_vec *v, const double *host_local);
/* VecAssemblyBegin/End: set_values writes owned entries immediately, so
 * assembly only completes the pending device work of the vector's stream. */
int kle_vec_assemble(kle_vec *v);
int kle_vec_ghost_update(kle_vec *v);                             /* halo fill  */
/* raw device pointer to the owned part (for zero-copy interop). */
int kle_vec_device_ptr(const kle_vec *v, double **dptr);

/* -------------------------------------------------------------------- mat */
/* Batch device assembly of the KLE system: replaces MatFS.build / buildFS
 * (mat_fs.py:131-192).  Produces node-block matrices K (dim x dim blocks),
 * Krhs (dim x dim) and Rw (dim x dim_w) with PETSc's pattern and ADD order. */
int kle_assemble_kle(kle_ctx *ctx, kle_mesh *m, kle_mat **K, kle_mat **Krhs, kle_mat **Rw);
/* Element matrices of local element e in tensor order (parity tests):
 * K_e [dim n][dim n], Rw_e [dim n][dim_w n] (row-major, n = ngl^dim). */
int kle_element_kle(kle_ctx *ctx, kle_mesh *m, int64_t e, double *Ke, double *Rwe);
/* No-slip assembly (replaces MatNS.build / buildNS, mat_ns.py:47-161):
 * K, Krhs, Rw as kle_assemble_kle on the no-slip nodes, Rd (free rows x
 * cell nodes), plus Kfs, Krhsfs, Rwfs, Rdfs with PETSc's DoF-level patterns,
 * and Ksum = K + Kfs (the operator of KleSolver.solverFS, kle_solver.py:22-28)
 * assembled directly. */
int kle_assemble_ns(kle_ctx *ctx, kle_mesh *m, kle_mat **K, kle_mat **Krhs, kle_mat **Rw, kle_mat **Rd,
                    kle_mat **Kfs, kle_mat **Krhsfs, kle_mat **Rwfs, kle_mat **Rdfs, kle_mat **Ksum);
/* Operators (replaces MatFS.buildOperators + Operators.setValues/assembleAll,
 * mat_fs.py:194-271, with Spectral.getElemKLEOperators spectral.py:162-228):
 * Curl [dim_w N x dim N], SrT [dim_s N x dim N], DivSrT [dim N x dim_s N],
 * each already scaled by the inverse lumped nodal weight.  Node-block CSR on
 * the full node adjacency (pattern 3), explicit zeros kept as PETSc does. */
int kle_assemble_operators(kle_ctx *ctx, kle_mesh *m, kle_mat **Curl, kle_mat **SrT, kle_mat **DivSrT);

/* Generic AIJ (petsc4py Mat().createAIJ + setValues + assemble). */
int kle_mat_create_aij(kle_ctx *ctx, int64_t m_local, int64_t n_local, int64_t m_global,
                       int64_t n_global, const int32_t *d_nnz, const int32_t *o_nnz,
                       kle_mat **out);
/* createAIJ(csr=(indptr, indices, data)): assembled scalar CSR (single rank),
 * strictly ascending columns per row. */
int kle_mat_create_aij_csr(kle_ctx *ctx, int64_t m, int64_t n, const int64_t *indptr, const int64_t *indices,
                           const double *data, kle_mat **out);
int kle_mat_set_values(kle_mat *A, int32_t nr, const int64_t *rows, int32_t nc,
                       const int64_t *cols, const double *v_rowmajor, int addv);
int kle_mat_assemble(kle_mat *A);
int kle_mat_destroy(kle_mat *A);
int kle_mat_get_size(const kle_mat *A, int64_t *m_global, int64_t *n_global);
int kle_mat_get_ownership_range(const kle_mat *A, int64_t *lo, int64_t *hi);
/* MatGetLocalSize (petsc4py Mat.getLocalSize; the local sizes behind
 * createVecLeft / createVecRight, base_problem.py:175,184, kle_solver.py:18) */
int kle_mat_get_local_size(const kle_mat *A, int64_t *m_local, int64_t *n_local);
int kle_mat_get_local_nnz(const kle_mat *A, int64_t *nnz);
/* MatGetInfo (+ sizes): PETSc nonzeros of the owned rows, the storage format
 * (0 node-block, 1 scalar AIJ), block shape and the SpMV's algorithmic bytes. */
typedef struct {
    int64_t m_global, n_global, m_local, n_local;
    int64_t nz_used;       /* PETSc nonzeros of the owned rows (explicit zeros included) */
    int format;            /* 0 node-block CSR, 1 scalar AIJ */
    int block_rows, block_cols;
    double spmv_bytes;     /* algorithmic bytes of one y = A x on this rank */
} kle_mat_info;
int kle_mat_get_info(const kle_mat *A, kle_mat_info *info);
int kle_mat_mult(kle_mat *A, kle_vec *x, kle_vec *y);            /* y = A x */
int kle_mat_mult_add(kle_mat *A, kle_vec *x, kle_vec *y, kle_vec *z); /* z = y + A x */
int kle_mat_diagonal_scale(kle_mat *A, const kle_vec *L, const kle_vec *R);
int kle_mat_get_diagonal(const kle_mat *A, kle_vec *d);
/* Y += a X where X's pattern is a subset of, or equal to, Y's. */
int kle_mat_axpy(kle_mat *Y, double a, const kle_mat *X);
int kle_mat_duplicate(const kle_mat *A, int copy_values, kle_mat **out);
/* Scalar CSR of the owned rows with GLOBAL column ids, PETSc pattern. */
int kle_mat_get_csr_size(const kle_mat *A, int64_t *m_local, int64_t *nnz);
/* Mat.getRow(row) (dmplex.py:332,363): owned global row -> global columns and
 * values in PETSc's pattern; call with cols = vals = NULL for the length. */
int kle_mat_get_row(const kle_mat *A, int64_t row, int64_t *ncols, int64_t *cols, double *vals);
int kle_mat_get_csr(const kle_mat *A, int64_t *indptr, int64_t *indices, double *data);
/* Convert (single rank) to the scalar-CSR device format (the AIJ kernel). */
int kle_mat_convert_aij(const kle_mat *A, kle_mat **out);
/* Structured columns: when every row's columns form a lattice box (K, Rw and
 * the operators on box meshes) the SpMV computes them from 8 B per row instead
 * of streaming 4 B per block (default on; 0 forces the column stream). */
int kle_mat_set_spmv_structured(kle_mat *A, int on);
int kle_mat_is_structured(const kle_mat *A, int *on);
/* Symmetric storage (MatSetOption(A, MAT_SPD, PETSC_TRUE) with PETSc's
 * MATSBAIJ layout; kle_solver.py:33-37 solves with the SPD K): keep only each
 * row's blocks from its diagonal block on and run the SpMV over them, every
 * stored off-diagonal block serving row i and, transposed, row j.  Needs a
 * 3x3 node-block matrix on a box lattice (one rank, or z slabs: the
 * transposed sums of upper ghost rows go back to their owner, MPISBAIJ's
 * reverse scatter) whose blocks are symmetric (to 1e-12 of the largest
 * entry; across ranks checked by one product through both storages);
 * otherwise KLE_ERR_SUP.  Collective at N > 1.  The full
 * storage stays (getRow, CSR export); any value change (diagonalScale, axpy,
 * setValues/assemble) drops the symmetric copy.  kle_assemble_kle turns it on
 * for K (tuning "spmv_sym", "spmv_sym_min_rows").  Results agree with the
 * full-storage SpMV to rounding (a different summation order); with the
 * default "spmv_sym_det" they are bitwise reproducible run to run. */
int kle_mat_set_symmetric(kle_mat *A, int on);
int kle_mat_get_symmetric(const kle_mat *A, int *on);
/* The brick decomposition of A's symmetric storage (kle_brick.hip; 0 bricks:
 * none -- full storage, tiles or the graph kernel): bricks, bricks along
 * x / y / z, region entries per row, the planner's modelled product time
 * (us). */
/* Diagnostic: move the symmetric storage's value array.  fresh = 1: to a new
 * allocation, `shift` bytes (a multiple of 8, <= 1 GiB) into it (the old one
 * freed).  fresh = 0: `shift` bytes into the allocation of the previous
 * fresh = 0 move -- the same physical pages, another offset (the first such
 * call makes that allocation, with 8 MB of room, at offset 0).  The product
 * is unchanged bit for bit; its speed should not depend on the offset
 * (tests/test_gpu_fullsize.py). */
int kle_mat_move_values(kle_mat *A, long long shift, int fresh);
int kle_mat_get_sym_bricks(const kle_mat *A, int *nbricks, int *dims, double *entries_per_row, double *model_us);
/* N > 1: run the rows that read no ghost entry while the halo exchange is in
 * flight on a second stream (default on). */
int kle_mat_set_halo_overlap(kle_mat *A, int on);
/* Row padding quantum (in blocks) of node-block matrices created afterwards:
 * every value stream of a row starts on a multiple of `quantum` doubles
 * (16 = one 128-B line) so adjacent streams never share a cache line. */
int kle_set_nb_pad(int quantum);  /* default 16 */
int kle_get_nb_pad(void);
/* Value layout of node-block matrices created afterwards: 0 = each row's
 * R*C value streams padded to the pad quantum; 1 = 16-block chunks (each
 * stream's 128-B line per chunk) + packed tail, rows 128-B aligned (no
 * per-stream padding). */
int kle_set_nb_layout(int layout);
int kle_get_nb_layout(void);
/* "nb" (node-block) or "aij". */
int kle_mat_get_format(const kle_mat *A, char *buf, int buflen);
/* Bytes one SpMV with this matrix moves (algorithmic: matrix + x + y). */
int kle_mat_spmv_bytes(const kle_mat *A, double *bytes);
/* Name of the kernel(s) y = A x launches with the current tuning, as rocprof
 * lists them (profile summaries, bench.py's roofline record). */
int kle_mat_spmv_kernel(const kle_mat *A, char *buf, int buflen);
/* Average device time (ms) of `reps` rank-local products y = A x: the bricks
 * and the gather of every row they touch, with no halo exchange either way
 * (the ghost x as they are).  A part's own kernel time, free of its
 * neighbours -- ranks that share a GPU take turns.  Box-brick symmetric
 * storage only (KLE_ERR_ARG otherwise); y's ghost-row sums are not sent. */
int kle_mat_time_local_spmv(kle_mat *A, const kle_vec *x, kle_vec *y, int reps, double *ms);

/* -------------------------------------------------------------------- ksp */
int kle_ksp_create(kle_ctx *ctx, kle_ksp **out);
int kle_ksp_destroy(kle_ksp *k);
int kle_ksp_set_type(kle_ksp *k, const char *type);      /* "cg" | "gmres" | "preonly" */
int kle_ksp_set_pc_type(kle_ksp *k, const char *type);   /* "none" | "jacobi" | "lu"   */
int kle_ksp_set_pc(kle_ksp *k, const char *type);        /* KSPSetPC(PCSetType): same as set_pc_type */
int kle_ksp_set_tolerances(kle_ksp *k, double rtol, double atol, double dtol, int maxit);
int kle_ksp_set_gmres_restart(kle_ksp *k, int restart);
/* CG with one reduction per iteration (Chronopoulos-Gear), as PETSc's
 * -ksp_cg_single_reduction. */
int kle_ksp_set_cg_single_reduction(kle_ksp *k, int flag);
/* Run exactly n iterations, no convergence test (benchmarks); 0 = off. */
int kle_ksp_set_fixed_iterations(kle_ksp *k, int n);
/* Benchmarks: n more iterations of the preceding fixed-iteration solve's
 * recurrence on the same (b, x) -- no restart (single-reduction / pipelined
 * CG), so a timed region holds exactly n iterations. */
int kle_ksp_continue(kle_ksp *k, kle_vec *b, kle_vec *x, int n);
int kle_ksp_set_operators(kle_ksp *k, kle_mat *A);
int kle_ksp_set_up(kle_ksp *k);
int kle_ksp_solve(kle_ksp *k, kle_vec *b, kle_vec *x);
int kle_ksp_get_iteration_number(const kle_ksp *k, int *its);
/* Kernel name(s) of the products inside the last solve call, as rocprof lists
 * them: kle_mat_spmv_kernel's, or -- where the CG update gathers a split
 * box-brick product itself -- the brick kernel alone (one rank). */
int kle_ksp_get_product_kernel(const kle_ksp *k, char *buf, int buflen);
/* Algorithmic bytes one of those products moves (kle_mat_spmv_bytes, or the
 * bricks' own share of a split product: the region sums written, not read). */
int kle_ksp_get_product_bytes(const kle_ksp *k, double *bytes);
int kle_ksp_get_residual_norm(const kle_ksp *k, double *rnorm);
int kle_ksp_get_converged_reason(const kle_ksp *k, int *reason);
/* ||b - A x|| / ||b|| recomputed after the last solve. */
int kle_ksp_get_true_relative_residual(const kle_ksp *k, double *rel);
/* CG / pipelined CG stop on their recursive residual (KSPSolve,
 * kle_solver.py:35), which drifts from the true one (pipelined: 1.1-1.3e-10
 * at rtol 1e-10).  When the true residual misses rtol, up to n correction
 * solves A e = b - A x (same method) follow, so the solve meets rtol on the
 * true residual (the north star's "same residual as PETSc KSP within
 * 1e-10"); n = 0 stops on the recursive residual exactly as PETSc's KSPCG /
 * KSPPIPECG do.  Default 2 (kle_set_tuning "ksp_refine" for new KSPs). */
int kle_ksp_set_corrections(kle_ksp *k, int n);
/* Iterations of the last solve's correction solves (0: none ran).  They are
 * NOT in kle_ksp_get_iteration_number, and the converged reason and residual
 * norm stay the main solve's (PETSc's KSPGetIterationNumber /
 * KSPGetConvergedReason of the recursive stop); each correction has max_it of
 * its own. */
int kle_ksp_get_correction_iterations(const kle_ksp *k, int *its);
/* Converged reason of the last correction solve (0: none ran; < 0: it hit
 * max_it or broke down and the true residual may still miss rtol). */
int kle_ksp_get_correction_reason(const kle_ksp *k, int *reason);

/* ------------------------------------------------------------ diagnostics */
/* Streaming read/copy microbenchmark (HBM ceiling for the roofline). */
int kle_stream_copy_bench(kle_ctx *ctx, int64_t bytes, int reps, double *gbps);
/* mode 0: copy (read+write bytes counted), 1: read-only 32 B/lane non-temporal,
 * 2: read-only 8 B/lane non-temporal, 3: read-only 8 B/lane plain. */
int kle_stream_bench(kle_ctx *ctx, int64_t bytes, int reps, int mode, double *gbps);

#ifdef __cplusplus
}
#endif
#endif
