/*
 * qvq.h -- C ABI of the MI355X LBG vector-quantization engine (libqvq.so).
 *
 * This is the drop-in boundary for coodie/quant's hot path.  The reference has no FFI;
 * its plugin interface is C++:
 *
 *   AbstractQuantizer::quantize(const std::vector<Vector>& trainingSet, size_t n, VectorType eps)
 *       -> tuple<codebook, assignedCodeVector, distortion>        include/Quantizer.hpp:10-16
 *   getQuantizer(Quantizers)                                       include/Quantizer.hpp:20,
 *                                                                  src/Quantizer.cpp:146-155
 *   CompressedImage::compress(image, quantizer, colorSpace, w, h, eps, N)
 *       (times getBlocksAsVectorsFromImage + quantize)             src/Compressor.cpp:107-123
 *
 * The C++ layer in include/quant_amd/ (libquant_amd.so) re-exposes exactly that
 * interface on top of these entry points; INTEGRATION.md shows the binding.  Everything
 * here is plain C: pointers, sizes, status codes; no exceptions cross this boundary.
 *
 * Results: code-vector indices are bit-identical to the reference's (src/Quantizer.cpp:24-32:
 * nanoflann's kd-tree answer over the codebook the reference computes, whose centroids are Kahan
 * sums in ascending row order, src/Quantizer.cpp:59-87) on any rank count; the returned codebook
 * is the exact sum of each final cell's members rounded once and multiplied by fl(1/count) (the
 * reference's Kahan sum agrees to <= 1 ulp).
 */
#ifndef QVQ_H
#define QVQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QVQ_API __attribute__((visibility("default")))

typedef struct qvq_ctx qvq_ctx;

typedef enum {
    QVQ_OK = 0,
    QVQ_EINVAL = 1,       /* bad argument (sizes, null pointers, bits out of range) */
    QVQ_ENOMEM = 2,       /* device or host allocation failed */
    QVQ_EDEVICE = 3,      /* HIP runtime error, or no HIP device */
    QVQ_ECOMM = 4,        /* RCCL error */
    QVQ_EUNSUPPORTED = 5, /* training set the engine cannot sum exactly (see qvq_set_vectors) */
    QVQ_ESTATE = 6        /* call order violated (e.g. qvq_lbg before a training set) */
} qvq_status;

/* Colour spaces, numbered as the reference's enum class ColorSpaces
 * (include/ColorSpace.hpp:6).  Only NORMAL and SCALED map bytes to values the engine
 * can sum exactly; CIE1931 is rejected with QVQ_EUNSUPPORTED. */
enum { QVQ_CS_NORMAL = 0, QVQ_CS_SCALED = 1, QVQ_CS_CIE1931 = 2 };

/* Per-level / per-call timings filled by qvq_get_timings (device ms from HIP events
 * recorded around each level's search kernel on the context's stream). */
typedef struct {
    int levels;                 /* split levels run by the last qvq_lbg */
    double total_ms;            /* whole qvq_lbg, host wall */
    double assign_ms[32];       /* device time of the assignment kernel per level (exact mode: wall time) */
    double update_ms[32];       /* device time of the centroid-sum kernel per level (exact mode: wall time) */
    double other_ms[32];        /* rest of the level: recheck, kd-tree ties, reduce, finalize + tables */
    uint64_t flagged[32];       /* rows re-checked in fp64 per level */
    uint64_t host_ties[32];     /* exact fp64 ties per level, answered by the reference kd-tree
                                   traversal (device kernel; host only for trees too deep) */
    double wait_ms[32];         /* host wall waiting for the level's codebook (previous finalize) */
    double tree_ms[32];         /* host wall building the level's kd-tree image (overlaps the search) */
    int kahan_redo;             /* 1: a level's ties failed the speculative reference-rule check, and the
                                   quantize ran again with synchronous reference-bit levels */
    int tie_overflow;           /* levels whose tie rows exceeded the check's export (each forces the redo) */
    int kahan_relays;           /* several ranks: levels whose tie rows needed cells summed over every
                                   rank's rows (the chained Kahan sums at the end of the call) */
    double mean_ms;             /* device time of the mean kernel (qvq_set_timing(-3) only) */
} qvq_timings;

/* Context: one per GPU per host thread.  Owns device memory and one HIP stream. */
QVQ_API qvq_status qvq_create(int hip_device, qvq_ctx **out);
QVQ_API void qvq_destroy(qvq_ctx *ctx);
QVQ_API const char *qvq_last_error(const qvq_ctx *ctx);
QVQ_API const char *qvq_version(void);

/*
 * Training set, way 1: raw P6 rasters (host pointer, n_images x xSize x ySize x 3 bytes,
 * image-major), tiled on the device exactly as getBlocksAsVectorsFromImage
 * (src/Compressor.cpp:31-62): the raster is read as xSize rows of ySize pixels, columns
 * past ySize wrap into the next row, components past the end of the buffer are 0.
 * Blocks of image i follow all blocks of image i-1.
 */
QVQ_API qvq_status qvq_set_images(qvq_ctx *ctx, const uint8_t *rgb, uint32_t n_images, uint32_t xSize,
                                  uint32_t ySize, uint32_t bw, uint32_t bh, int colorspace);
/* Same, but the rasters are already in device memory (e.g. a torch tensor). */
QVQ_API qvq_status qvq_set_images_device(qvq_ctx *ctx, const void *d_rgb, uint32_t n_images, uint32_t xSize,
                                         uint32_t ySize, uint32_t bw, uint32_t bh, int colorspace);
/* Same, with the rasters generated on the device by the synthetic generator of
 * SURVEY.md 8(d) (image i uses seed0 + i); for benchmarks and scale tests. */
QVQ_API qvq_status qvq_set_synthetic(qvq_ctx *ctx, uint32_t S, uint64_t seed0, uint32_t n_images, uint32_t bw,
                                     uint32_t bh, int colorspace);
/*
 * Training set, way 2: flat fp64 N x dim (the AbstractQuantizer path, include/Quantizer.hpp:10-16).
 * When every value is one the NORMAL or SCALED colour space produces from a byte (or 0.0) the
 * fast path applies (exact integer sums: centroids within 1 ulp of the reference's Kahan sums).
 * Any other data (arbitrary finite doubles, CIE1931 values) takes the exact mode of
 * qvq_set_vectors_exact.
 */
QVQ_API qvq_status qvq_set_vectors(qvq_ctx *ctx, const double *X, uint64_t n, uint32_t dim);
/*
 * Training set in exact mode, any finite fp64 data: the reference's arithmetic bit for bit
 * -- fp64 search in nanoflann's order with kd-tree ties, centroids as the Kahan sum of each
 * cell's rows in ascending order times fl(1/n) (src/Quantizer.cpp:46-87), so codebook and
 * indices equal the reference's exactly.  Sequential Kahan chains make it slower than the
 * byte path; one rank only (QVQ_EUNSUPPORTED with a communicator).  n < 2^31.
 */
QVQ_API qvq_status qvq_set_vectors_exact(qvq_ctx *ctx, const double *X, uint64_t n, uint32_t dim);

QVQ_API uint64_t qvq_num_vectors(const qvq_ctx *ctx);
QVQ_API uint32_t qvq_dim(const qvq_ctx *ctx);

/*
 * Full split-LBG (LBGQuantizer::quantize, src/Quantizer.cpp:122-143) over the training
 * set: n = bits levels, K = 2^bits code vectors.  eps is accepted for signature parity;
 * it cannot change the outputs (one Lloyd step per level).
 * Outputs (caller-owned host memory, any may be NULL):
 *   codebook   : K x dim fp64
 *   assign     : n u32 (this rank's rows)
 *   distortion : mean squared error of the final codebook, as updateDistortion
 * With a communicator (qvq_comm_init) every rank runs this on its own rows -- consecutive ranges
 * of the global rows, rank 0 first -- and all ranks get the same codebook, distortion and indices
 * as one rank over all the rows (the reference's Kahan rule included: cells whose reference bits
 * decide a tie are summed across the ranks in row order).
 */
QVQ_API qvq_status qvq_lbg(qvq_ctx *ctx, uint32_t bits, double eps, double *codebook, uint32_t *assign,
                           double *distortion);
/* Device pointer to the last qvq_lbg's assignment (u32, qvq_num_vectors entries). */
QVQ_API const uint32_t *qvq_assign_device(const qvq_ctx *ctx);

/* Single steps over the current training set, for tests and benchmarks.
 * qvq_assign: nearest code vector of every row for codebook C (K x dim fp64, host),
 *   with the same MFMA/VALU search + fp64 recheck + kd-tree tie resolution as qvq_lbg.
 * qvq_update: centroids of the rows under assignment A (host, n u32) into C_out
 *   (K x dim fp64) and counts (K u64), the engine's exact-sum rule. */
QVQ_API qvq_status qvq_assign(qvq_ctx *ctx, const double *C, uint32_t K, uint32_t *assign);
QVQ_API qvq_status qvq_update(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, double *C_out, uint64_t *counts);
/* The reference's own centroid bits (Solution::fixCodeVectors, reference src/Quantizer.cpp:59-87:
 * Kahan sums in ascending row order times fl(1/n), empty cells 0) of the resident rows under
 * assignment A, into C_out (K x dim fp64).  With a communicator of several ranks every rank passes
 * its own rows' assignment and gets the centroids of all ranks' rows, each cell's chain running
 * over the ranks' rows in rank order (the ranks must hold consecutive ranges of the global rows,
 * rank 0 first, as qvq_lbg's sharding does). */
QVQ_API qvq_status qvq_update_kahan(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, double *C_out);
/* Test entry: qvq_update_kahan with this context's rows cut into nsplits virtual ranks at
 * splits[0..nsplits] (0 = splits[0] <= ... <= splits[nsplits] = N), the several-rank chained
 * evaluation run rank after rank on one device; equals qvq_update_kahan for any cuts. */
QVQ_API qvq_status qvq_update_kahan_split(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, const uint64_t *splits,
                                          uint32_t nsplits, double *C_out);

/* Decode (replaces CompressedImage::decompress, reference src/Compressor.cpp:156-165, and the
 * getImageFromVectors it calls, src/Compressor.cpp:64-85): raster[x*ySize+y] = the code-vector bytes
 * codebook[assign[block]] laid out as getImageFromVectors does, including the column wrap and
 * "last block wins" order.  codebook: K x (bw*bh*3) bytes; assign: ceil(xSize/bw)*ceil(ySize/bh)
 * u32; rgb: xSize*ySize*3 bytes.  An index >= K returns QVQ_EINVAL (the reference indexes
 * codeVectors with operator[], undefined behaviour).  ySize + bh - 1 and xSize + bw - 1 must be
 * below 2^32.
 * qvq_decode takes host buffers.  qvq_decode_mse also returns the raport's distortion, the mean
 * squared difference of the signed bytes of orig and the decoded raster (src/Compressor.cpp:
 * 133-146), computed in the same device pass (rgb may then be NULL).  qvq_decode_device takes
 * device pointers and a hipStream_t on which it launches (NULL = the legacy null stream, so
 * work the caller queued on blocking streams is ordered before it; the engine's own queued work
 * is ordered before it on any stream) and synchronises that stream before returning.  d_assign
 * must be 4-byte aligned (QVQ_EINVAL otherwise); an unaligned raster takes a per-pixel kernel,
 * as does the host qvq_decode path for any alignment of its staging. */
QVQ_API qvq_status qvq_decode(qvq_ctx *ctx, const uint8_t *codebook, uint32_t K, const uint32_t *assign,
                              uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh, uint8_t *rgb);
QVQ_API qvq_status qvq_decode_mse(qvq_ctx *ctx, const uint8_t *codebook, uint32_t K, const uint32_t *assign,
                                  uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh,
                                  uint8_t *rgb, const uint8_t *orig, double *mse);
QVQ_API qvq_status qvq_decode_device(qvq_ctx *ctx, const void *d_codebook, uint32_t K, const void *d_assign,
                                     uint64_t nblocks, uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh,
                                     void *d_rgb, void *stream);

/* Multi-GPU: join an RCCL communicator (unique_id from qvq_comm_unique_id on rank 0,
 * shipped to the other ranks by the caller).  Each level then all-reduces the
 * per-code-vector sums and counts over xGMI.  nranks = 1 creates a real one-rank
 * communicator (the collective path with identical results).  A collective that fails, or
 * a wait that outlasts the timeout (qvq_set_timeout) while a communicator is joined, returns
 * QVQ_ECOMM and aborts the communicator (the context then runs single-rank until the next
 * qvq_comm_init). */
QVQ_API qvq_status qvq_comm_unique_id(uint8_t id[128]);
QVQ_API qvq_status qvq_comm_init(qvq_ctx *ctx, int nranks, int rank, const uint8_t id[128]);
/* Test-only communicator: every per-level exchange (the same buffers the RCCL all-reduce
 * sums: the mean's and the level's per-code-vector sums and counts as u64, dtype 0; the two
 * distortion terms as double, dtype 1) is copied to pinned host memory, fn(buf, count, dtype,
 * user) must replace it in place by the sum over the nranks ranks and return 0, and the
 * result is copied back.  Lets several processes share one GPU (RCCL refuses two ranks on one
 * device) so the sharded schedule runs in tests on a one-GPU box.  Replaces any communicator. */
typedef int (*qvq_allreduce_fn)(void *buf, uint64_t count, int dtype, void *user);
QVQ_API qvq_status qvq_comm_init_host(qvq_ctx *ctx, int nranks, int rank, qvq_allreduce_fn fn, void *user);
/* The joined communicator: ranks, this rank, kind (QVQ_COMM_NONE: single rank). */
enum { QVQ_COMM_NONE = 0, QVQ_COMM_RCCL = 1, QVQ_COMM_HOST = 2 };
QVQ_API qvq_status qvq_comm_info(const qvq_ctx *ctx, int *nranks, int *rank, int *kind);
/* Bound, in seconds, of every host wait on the context's stream (default 120, or the
 * QVQ_TIMEOUT_S environment variable at qvq_create).  A wait that fails while the stream
 * cannot be drained poisons the context: results are never copied into caller memory after
 * the call returned, and every later call but qvq_destroy returns QVQ_ESTATE. */
QVQ_API qvq_status qvq_set_timeout(qvq_ctx *ctx, double seconds);

/* Which levels get HIP events around their search kernel (each event record idles the GPU
 * ~6 us: every level costs ~10 % of a C3 quantize): -1 every level, -2 none (default), -3 the
 * mean kernel only (mean_ms), n >= 0 level n+1 only.  Unmeasured levels report 0 in
 * qvq_get_timings. */
QVQ_API qvq_status qvq_set_timing(qvq_ctx *ctx, int level);
QVQ_API qvq_status qvq_get_timings(const qvq_ctx *ctx, qvq_timings *out);

/* Test entry: the reference kd-tree of C (K x dim fp64) built on the device (the build qvq_lbg
 * uses for its 48-D levels) against the host's RefKDTree, node for node; result 0 equal, 1
 * different (qvq_last_error names the first difference), 2 the device build gave up.  build_ms
 * (4 doubles): the launch, then its phases (big nodes, small subtrees, the images). */
QVQ_API qvq_status qvq_kdtree_device_check(qvq_ctx *ctx, const double *C, uint32_t K, uint32_t dim, double *build_ms,
                                           uint32_t *result);

/* Host-only helpers (no GPU needed), exported for tests of the host logic. */
/* The reference kd-tree's answer for nq queries (nanoflann semantics, see kdtree.hpp). */
QVQ_API qvq_status qvq_host_kdtree_nn(const double *C, uint32_t K, uint32_t dim, const double *Q, uint64_t nq,
                                      uint32_t *out);
/* The host kd-tree build over C (K x dim), as the device build's image (kdtree_dev.hpp
 * kdb_host_layout: header | nodes[2K], breadth first | point boxes [2K][lo D | hi D] | vind[K]);
 * *need = the image's bytes, written when bytes >= *need (QVQ_EINVAL otherwise).  For tests of
 * the build against a restatement, node for node. */
QVQ_API qvq_status qvq_host_kdtree_image(const double *C, uint32_t K, uint32_t dim, void *img, uint64_t bytes,
                                         uint64_t *need);
/* Exact centroid finalisation from reduced sums, as the device does it:
 * C[k][d] = round(R*hi + lo - bias*cnt) * 2^-scale * fl(1/cnt).  For tests. */
QVQ_API qvq_status qvq_host_finalize(const uint64_t *hi, const uint64_t *lo, const uint64_t *cnt, uint32_t K,
                                     uint32_t dim, int colorspace, double *C_out);
/* Per-block exact contributions of one row of codes, as the device sums them: hi/lo
 * (dim entries each) -- for the host-side sharding tests. */
QVQ_API qvq_status qvq_host_row_terms(const uint8_t *codes, uint32_t dim, int colorspace, uint64_t *hi,
                                      uint64_t *lo);
/* The engine's bounded-wait policy (quant_amd/csrc/wait.hpp) driven by scripted probes, for
 * tests: scenario 0 the work publishes after ~5 ms; 1 it never does, no communicator; 2 it
 * never does, a healthy communicator; 3 the communicator reports an error after ~5 ms; 4 the
 * stream fails; 5 the stream drains without publishing.  Returns the wait's status and its
 * duration in *elapsed_s. */
QVQ_API qvq_status qvq_host_wait_probe(int scenario, double timeout_s, double *elapsed_s);
/* The certificate's helper-thread pool (engine.cpp pool_run) over `rounds` jobs of 1..maxn (<= 64)
 * threads, the count changing from job to job: *errors = job slots that ran other than exactly
 * once.  Host only, for tests. */
QVQ_API qvq_status qvq_host_pool_stress(uint32_t rounds, uint32_t maxn, uint64_t *errors);

#ifdef __cplusplus
}
#endif
#endif /* QVQ_H */
