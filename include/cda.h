/*
 * cda.h -- C ABI of libcda.so, the MI355X (gfx950) implementation of
 * celestia-app's block data-availability hot path:
 *
 *   ODS (k x k shares of 512 B) -> EDS (2k x 2k, Leopard RS) -> 4k NMT
 *   row/column roots -> DataAvailabilityHeader data root.
 *
 * Every entry point replaces one reference interface (paths relative to the
 * celestia-app v3 tree; EXT = third-party Go module pinned in go.mod):
 *
 *   cda_extend_shares      da.ExtendShares            pkg/da/data_availability_header.go:65-75
 *   cda_dah_from_eds       da.NewDataAvailabilityHeader pkg/da/data_availability_header.go:44-63
 *                          (+ rsmt2d (*EDS).RowRoots/ColRoots via
 *                          wrapper.NewConstructor, pkg/wrapper/nmt_wrapper.go:73-86)
 *   cda_extend_dah         ExtendShares + NewDataAvailabilityHeader in one
 *                          submission (app/prepare_proposal.go:61,71;
 *                          app/process_proposal.go:138,144)
 *   cda_extend_dah_batch   the same for n independent squares
 *   cda_rs_encode          rsmt2d Codec.Encode (appconsts.DefaultCodec,
 *                          pkg/appconsts/global_consts.go:92 -> LeoRSCodec)
 *   cda_data_root          (*DataAvailabilityHeader).Hash
 *                          pkg/da/data_availability_header.go:92-108
 *   cda_extend_dah_device  device-resident batch (inputs/outputs in HBM)
 *   cda_extend_dah_inplace_device
 *                          the same with the ODS already in Q0 of the EDS
 *                          (rsmt2d ImportExtendedDataSquare-style arena)
 *   cda_square_layout / cda_square_construct / cda_construct_extend_dah /
 *   cda_square_construct_device
 *                          go-square square.Construct / square.Build (EXT
 *                          v1.1.0, go.mod:9; app/process_proposal.go:122,
 *                          app/prepare_proposal.go:50, app/extend_block.go:16)
 *   cda_blob_commitments   go-square inclusion.CreateCommitment
 *                          (x/blob/types/blob_tx.go:98, payforblob.go:53)
 *   cda_repair             rsmt2d ExtendedDataSquare.Repair (EXT v0.14.0)
 *   cda_rs_decode          rsmt2d Codec.Decode (reedsolomon Reconstruct)
 *   cda_square_*           resident squares: proof.NewShareInclusionProofFromEDS
 *                          (pkg/proof/proof.go:77), inclusion.GetCommitment
 *                          (pkg/inclusion/get_commit.go:12)
 *   cda_nmt_axis_root(s) / cda_nmt_prove_range
 *                          wrapper.NewErasuredNamespacedMerkleTree + Push +
 *                          Root / ProveRange (pkg/wrapper/nmt_wrapper.go:55-129)
 *   cda_merkle_root        go-square/merkle HashFromByteSlices (DAH.Hash for
 *                          any root count, data_availability_header.go:92-108)
 *   cda_comm_* / cda_extend_dah_split / cda_extend_dah_multi
 *                          multi-GPU configs 4 and 5 (app/process_proposal.go:138-152
 *                          block replay; one square over G GPUs)
 *
 * Conventions
 *   - All buffers are plain byte arrays; shares are row-major and contiguous
 *     (share (r, c) of a width-w square at offset (r*w + c)*512).  NMT roots
 *     are 90 bytes (min ns 29 || max ns 29 || sha256 32), packed.
 *   - Inputs are borrowed for the duration of the call; outputs are written to
 *     caller-owned buffers; the library keeps no pointer after return.
 *   - Return value: CDA_OK (0) or a negative CDA_ERR_* code.  The message of
 *     the calling thread's last call is available from cda_last_error(); it
 *     uses the reference's error text where one exists.  The library never
 *     aborts across the ABI.
 *   - A context owns one HIP device and stream; calls on one context are
 *     serialised by an internal mutex (rsmt2d calls Codec/Tree from many
 *     goroutines) and may come from any OS thread (the context's device is
 *     made current for the call).  Device entry points only enqueue on the
 *     caller's stream; their GPU work is ordered after the previous call's on
 *     the same context (any stream), because the context's scratch is shared.
 *     Use one context per device.
 */
#ifndef CDA_H
#define CDA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CDA_SHARE_SIZE 512     /* appconsts.ShareSize, pkg/appconsts/global_consts.go:29 */
#define CDA_NAMESPACE_SIZE 29  /* appconsts.NamespaceSize, global_consts.go:26 */
#define CDA_NMT_ROOT_SIZE 90   /* 2*NamespaceSize + sha256.Size */
#define CDA_HASH_SIZE 32

enum {
    CDA_OK = 0,
    CDA_ERR_NOT_POW2 = -1,      /* "number of shares is not a power of 2: got %d" (data_availability_header.go:68) */
    CDA_ERR_CHUNK_SIZE = -2,    /* rsmt2d LeoRSCodec.ValidateChunkSize: "chunkSize %v must be a multiple of 64 bytes" */
    CDA_ERR_PUSH_ORDER = -3,    /* nmt ErrInvalidPushOrder on a Q0 row/column (surfaces from RowRoots/ColRoots) */
    CDA_ERR_DEVICE = -4,        /* HIP runtime / kernel launch failure */
    CDA_ERR_OOM = -5,           /* device allocation failure */
    CDA_ERR_INVALID = -6,       /* bad argument (NULL pointer, k out of range, ...) */
    CDA_ERR_UNSUPPORTED = -7,   /* shard count the codec does not support */
    CDA_ERR_SQUARE = -8,        /* go-square square.Construct / Build error (message from cda_last_error) */
    CDA_ERR_BYZANTINE = -9,     /* rsmt2d ErrByzantineData ("byzantine row: %d" / "byzantine col: %d") */
    CDA_ERR_UNREPAIRABLE = -10, /* rsmt2d ErrUnrepairableDataSquare ("failed to solve data square") /
                                   reedsolomon ErrTooFewShards */
    CDA_ERR_COMM = -11          /* an RCCL call failed: the context's communicator was aborted and
                                   released; every rank must call cda_comm_init again */
};

typedef struct cda_ctx cda_ctx;

/* Context lifecycle. device: HIP ordinal (-1 = current device). */
int cda_ctx_create(int device, cda_ctx **out);
int cda_ctx_destroy(cda_ctx *ctx);
/* Message of the calling thread's last call (never NULL; "" after success).
 * Thread-local, so a concurrent call on the same context from another thread
 * cannot change or free it; a cgo caller reads it in the same C call or under
 * runtime.LockOSThread. */
const char *cda_last_error(cda_ctx *ctx);
/* Library version string, e.g. "cda 0.1.0 gfx950". */
const char *cda_version(void);

/* da.ExtendShares: ods = k*k*512 bytes (k a power of two, k >= 1);
 * eds = (2k)^2*512 bytes. n_shares is len(s) (checked for power of two). */
int cda_extend_shares(cda_ctx *ctx, const uint8_t *ods, uint32_t n_shares, uint8_t *eds);

/* da.NewDataAvailabilityHeader on an existing EDS of width w = 2k:
 * row_roots, col_roots = w*90 bytes each; data_root = 32 bytes (DAH.Hash()).
 * Returns CDA_ERR_PUSH_ORDER if a Q0 row or column is not namespace ordered. */
int cda_dah_from_eds(cda_ctx *ctx, const uint8_t *eds, uint32_t w, uint8_t *row_roots, uint8_t *col_roots,
                     uint8_t *data_root);

/* ExtendShares + NewDataAvailabilityHeader in one device submission. eds may be
 * NULL when the caller only needs the roots. On CDA_ERR_PUSH_ORDER the EDS is
 * still written (ExtendShares succeeds; the error belongs to the DAH step), and
 * so are the roots and data root: those of the reference's fraud tooling,
 * NewDataAvailabilityHeader over test/util/malicious/tree.go's BlindTrees (no
 * order check; the hashing never depends on it).  The same holds per square in
 * the batch entry points. */
int cda_extend_dah(cda_ctx *ctx, const uint8_t *ods, uint32_t n_shares, uint8_t *eds, uint8_t *row_roots,
                   uint8_t *col_roots, uint8_t *data_root);

/* Batch of n squares of width k, contiguous: ods = n*k*k*512, eds = n*(2k)^2*512
 * (or NULL), row_roots/col_roots = n*2k*90, data_roots = n*32. status (may be
 * NULL) receives one CDA_OK / CDA_ERR_PUSH_ORDER per square; the call returns
 * CDA_ERR_PUSH_ORDER if any square failed. */
int cda_extend_dah_batch(cda_ctx *ctx, const uint8_t *ods, uint32_t k, uint32_t n, uint8_t *eds, uint8_t *row_roots,
                         uint8_t *col_roots, uint8_t *data_roots, int32_t *status);

/* cda_extend_dah_batch with a choice of what goes back into eds (NULL: roots
 * only, as before):
 *   CDA_EDS_FULL     eds = n*(2k)^2*512, the whole EDS (= cda_extend_dah_batch);
 *                    the library copies Q0 from ods on host threads;
 *   CDA_EDS_SKIP_Q0  the same buffer, Q0 left untouched: a cgo caller that
 *                    wraps the EDS with rsmt2d.ImportExtendedDataSquare points
 *                    the Q0 cells at its own shares (it holds them already),
 *                    which saves the host copy of Q0;
 *   CDA_EDS_PARITY   eds = n*3*k^2*512 packed parity: per square Q1 as k rows
 *                    of k shares ([k][k][512]), then EDS rows k..2k-1 whole
 *                    ([k][2k][512]); Q0 is the caller's ODS.  The device packs
 *                    each chunk and returns it in one linear copy.
 * Reference: pkg/da/data_availability_header.go:65-75 (ExtendShares returns
 * the EDS whose Q0 cells are the input shares). */
#define CDA_EDS_FULL 0
#define CDA_EDS_SKIP_Q0 1
#define CDA_EDS_PARITY 2
int cda_extend_dah_batch_ex(cda_ctx *ctx, const uint8_t *ods, uint32_t k, uint32_t n, uint8_t *eds, int eds_mode,
                            uint8_t *row_roots, uint8_t *col_roots, uint8_t *data_roots, int32_t *status);

/* Device-resident batch: every pointer is device memory on ctx's device;
 * stream is a hipStream_t; NULL is HIP's default (null) stream, the one a
 * PyTorch/Go caller enqueues on by default -- NOT the context's private
 * stream, so the call is ordered after the caller's own work. Asynchronous: the
 * call only enqueues work. Per-square push-order status is written to d_status
 * (n int32, device memory, may be NULL). */
int cda_extend_dah_device(cda_ctx *ctx, const void *d_ods, uint32_t k, uint32_t n, void *d_eds, void *d_row_roots,
                          void *d_col_roots, void *d_data_roots, int32_t *d_status, void *stream);

/* Size the context's scratch for device batches of up to n squares of width
 * k (synchronous).  Scratch buffers only grow; inside a call a growing buffer
 * is released and reallocated in stream order on the call's stream
 * (hipFreeAsync / hipMallocAsync: no device synchronisation), so device entry
 * points stay enqueue-only either way; cda_reserve just moves the allocations
 * out of the first calls. */
int cda_reserve(cda_ctx *ctx, uint32_t k, uint32_t n);

/* As cda_extend_dah_device, but the k*k ODS shares are already in place in
 * quadrant Q0 of d_eds (row r, column c at (r*2k + c)*512 of each square),
 * the layout rsmt2d's EDS has after ExtendShares.  The cgo caller flattens the
 * [][]byte shares straight into that arena (it must copy them into one flat
 * buffer anyway), so the kernels read Q0 where it lies and never copy it.
 * Outputs and semantics are identical to cda_extend_dah_device. */
int cda_extend_dah_inplace_device(cda_ctx *ctx, uint32_t k, uint32_t n, void *d_eds, void *d_row_roots,
                                  void *d_col_roots, void *d_data_roots, int32_t *d_status, void *stream);

/* rsmt2d Codec.Encode (Leopard, GF(2^8) for 2*n_shards <= 256, else GF(2^16)):
 * n_codewords codewords, each n_shards data shards of shard_len bytes,
 * contiguous; parity has the same shape. n_shards a power of two. */
int cda_rs_encode(cda_ctx *ctx, const uint8_t *data, uint32_t n_shards, uint32_t shard_len, uint32_t n_codewords,
                  uint8_t *parity);

/* (*DataAvailabilityHeader).Hash: RFC-6962 root of row_roots || col_roots
 * (w roots of 90 bytes each). w == 0 gives sha256("") like Hash() on a nil DAH. */
int cda_data_root(cda_ctx *ctx, const uint8_t *row_roots, const uint8_t *col_roots, uint32_t w, uint8_t *data_root);

/* Details of the calling thread's last CDA_ERR_PUSH_ORDER: axis (0 row, 1
 * column), the axis index, and the leaf position whose push failed. */
int cda_push_order_detail(cda_ctx *ctx, int32_t *axis, uint32_t *index, uint32_t *position);
/* The same detail for square `square` of the context's last device batch
 * (cda_extend_dah_device / cda_extend_dah_inplace_device), whose d_status
 * carries only CDA_ERR_PUSH_ORDER: waits for that batch's GPU work, then
 * decodes the square's first violation (axis -1 when the square is ordered).
 * Valid until the next device batch on the context.  A block-replay caller
 * (app/process_proposal.go:138-147) builds the rejection text from it. */
int cda_push_order_detail_at(cda_ctx *ctx, uint32_t square, int32_t *axis, uint32_t *index, uint32_t *position);

/* Config 5: ONE square split across G ranks (one GPU each), row blocks +
 * column blocks.  k = ODS width, W = 2k, R = k/G rows and C = W/G columns per
 * rank.  All pointers are device memory; calls only enqueue on `stream`
 * (NULL = HIP's default stream, as for cda_extend_dah_device).
 * d_err is one uint32 per rank, initialised by the caller to 0xFFFFFFFF;
 * push-order violations atomically lower it (encoding: axis<<24 | index<<12 |
 * position, reduce with MIN across ranks).
 *  1. cda_split_rows: ODS rows [row0, row0+R) (R x k shares, row-major) ->
 *     row block (R x W shares: Q0 row | Q1 row), plus the Q0 row-order check.
 *  2. caller: all-to-all of the row blocks' column slices (RCCL) so rank g
 *     holds rows 0..k-1 of columns [g*C, g*C+C) as a W x C share block.
 *  3. cda_split_cols: column-encode the block (Q0->Q2 / Q1->Q3), hash each
 *     cell once, write the C column roots and, per EDS row, the NMT subtree
 *     node over this rank's C columns (96-B slots, W of them).
 *  4. caller: gather the subtree slots ([G][W][96]) and column root slots
 *     ([W][96], rank order) on one rank.
 *  5. cda_split_combine: top log2(G) levels of every row tree, pack roots,
 *     data root. */
int cda_split_rows(cda_ctx *ctx, const void *d_ods_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                   void *d_row_block, uint32_t *d_err, void *stream);
int cda_split_cols(cda_ctx *ctx, void *d_col_block, uint32_t k, uint32_t n_cols, uint32_t col0,
                   void *d_col_root_slots, void *d_row_subtree_slots, uint32_t *d_err, void *stream);
int cda_split_combine(cda_ctx *ctx, const void *d_row_subtree_slots, uint32_t parts, uint32_t k,
                      const void *d_col_root_slots, void *d_row_roots, void *d_col_roots, void *d_data_root,
                      void *stream);

/* ---- Multi-GPU inside the library ---------------------------
 * Config 5 with the library's own RCCL collectives (no torch.distributed in the
 * host): rank 0 makes an id (cda_comm_unique_id, 128 bytes) and hands it to
 * every rank out of band; each rank's context joins (cda_comm_init, one context
 * per GPU, all ranks call it together); cda_extend_dah_split then runs the
 * whole split of ONE square on `stream`: rows into the all-to-all send layout,
 * a grouped ncclSend/ncclRecv all-to-all, column encode + hashing, a gather of
 * the subtree / column-root slots and a MIN reduce of the push-order word to
 * rank 0, which writes the roots and the data root.  Every rank must call it.
 *   d_ods_rows: this rank's R = k/G ODS rows (R*k shares, device);
 *   d_col_block: W x C shares (device, may be NULL = library scratch): the EDS
 *     columns [rank*C, rank*C + C) on return (row-major [W][C][512]);
 *   d_row_roots / d_col_roots (W*90) / d_data_root (32): rank 0 only;
 *   d_err: one device uint32, on rank 0 the MIN over ranks of the push-order
 *     words (0xFFFFFFFF = ordered; axis<<24 | index<<12 | position; 0 = a rank
 *     failed locally: rank 0 then returns CDA_ERR_DEVICE and writes no roots). */
#define CDA_COMM_ID_BYTES 128
int cda_comm_unique_id(uint8_t id[CDA_COMM_ID_BYTES]);
int cda_comm_init(cda_ctx *ctx, int rank, int world, const uint8_t id[CDA_COMM_ID_BYTES]);
int cda_comm_destroy(cda_ctx *ctx);
/* The live communicator's rank and rank count as RCCL formed them
 * (ncclCommUserRank / ncclCommCount); CDA_ERR_INVALID without one. */
int cda_comm_size(cda_ctx *ctx, int *rank, int *world);
/* ncclCommAbort of the context's communicator (then released).  Takes no
 * context lock, so a host watchdog may call it from another thread while a
 * call on the context waits in a collective for a peer that failed.  Errors
 * of cda_extend_dah_split: checks that depend on k / the world size fail on
 * every rank before any collective; scratch is sized when k changes, followed
 * by one agreement all-reduce, so an allocation failure on any rank makes
 * every rank return CDA_ERR_OOM; a local failure after that keeps the rank in
 * the remaining collectives with its push-order word poisoned to 0 and returns
 * the rank's error; rank 0 reads the reduced word back and, when it is 0 (a
 * peer failed), returns CDA_ERR_DEVICE without writing roots; a failed RCCL
 * call closes its group, aborts the communicator and returns CDA_ERR_COMM, and
 * so does a call that cda_comm_abort released while it waited in a collective
 * (every RCCL post re-reads the communicator under a lock that the abort also
 * takes, so no call touches an aborted communicator). */
int cda_comm_abort(cda_ctx *ctx);
int cda_extend_dah_split(cda_ctx *ctx, const void *d_ods_rows, uint32_t k, void *d_col_block, void *d_row_roots,
                         void *d_col_roots, void *d_data_root, uint32_t *d_err, void *stream);
/* Step 1 of the split for a caller that runs its own all-to-all (e.g. over
 * torch.distributed): the row block of R ODS rows written straight in the send
 * layout [parts][R][C][512] (part h = columns [h*C, h*C + C)), so the received
 * pieces ARE rows 0..k-1 of the receiver's column block. */
int cda_split_rows_send(cda_ctx *ctx, const void *d_ods_rows, uint32_t k, uint32_t n_rows, uint32_t row0,
                        uint32_t parts, void *d_send, uint32_t *d_err, void *stream);
/* The split's buffer arithmetic (host only, no context; csrc/split_layout.h,
 * the same functions the group-rows kernel and cda_extend_dah_split use), so a
 * host can size its buffers and a test can replay the G > 1 exchange on the
 * CPU.  Byte sizes / offsets: the all-to-all piece of one rank pair, the send
 * buffer [G][R][C][512], the column block [W][C][512], and in the slot area
 * (96-B NMT node slots) the rank's C column roots, its W row subtree nodes,
 * (rank 0) the gathered [G][W] subtrees and [W] column roots, the push-order
 * word.  CDA_ERR_INVALID unless k and world are powers of two, world | k. */
typedef struct {
    uint32_t k, world, W, R, C;
    uint64_t piece_bytes, send_bytes, col_block_bytes;
    uint64_t col_slots_off, row_sub_off, gather_sub_off, gather_col_off, err_off, slots_bytes;
} cda_split_layout_t;
int cda_split_layout(uint32_t k, uint32_t world, cda_split_layout_t *out);
/* n offsets at once, off[i] for (a[i], b[i]) (b may be NULL when unused):
 *   CDA_SPLIT_SEND        send-buffer byte offset of row-block cell (r = a, col = b)
 *   CDA_SPLIT_SEND_PIECE  send-buffer byte offset of the piece for rank a
 *   CDA_SPLIT_RECV_PIECE  column-block byte offset where rank a's piece lands
 *   CDA_SPLIT_BLOCK       column-block byte offset of EDS row a, local column b
 *   CDA_SPLIT_GATHER_SUB  slot-area byte offset of rank a's W row subtrees (rank 0)
 *   CDA_SPLIT_GATHER_COL  slot-area byte offset of rank a's C column roots (rank 0)
 *   CDA_SPLIT_COMBINE     slot index, in the gathered subtrees, of rank a's node of row b
 * CDA_ERR_INVALID (nothing written) for an unknown kind, an index out of its
 * range (r < R, col < W, row < W, c < C, ranks < world) or b NULL where read. */
#define CDA_SPLIT_SEND 0
#define CDA_SPLIT_SEND_PIECE 1
#define CDA_SPLIT_RECV_PIECE 2
#define CDA_SPLIT_BLOCK 3
#define CDA_SPLIT_GATHER_SUB 4
#define CDA_SPLIT_GATHER_COL 5
#define CDA_SPLIT_COMBINE 6
int cda_split_offsets(uint32_t k, uint32_t world, int what, uint32_t n, const uint32_t *a, const uint32_t *b,
                      uint64_t *off);
/* Config 4 on one node: n independent squares (host buffers, as
 * cda_extend_dah_batch) split into contiguous shards over n_ctx contexts (one
 * per GPU) and run concurrently on host threads; no collective. */
int cda_extend_dah_multi(cda_ctx *const *ctxs, uint32_t n_ctx, const uint8_t *ods, uint32_t k, uint32_t n,
                         uint8_t *eds, uint8_t *row_roots, uint8_t *col_roots, uint8_t *data_roots, int32_t *status);

/* ---- Data-square construction ----------------------
 * go-square v1.1.0 square.Construct (mode CDA_SQUARE_CONSTRUCT; used by
 * ProcessProposal app/process_proposal.go:122-126 and ExtendBlock
 * app/extend_block.go:16-20) and square.Build (mode CDA_SQUARE_BUILD;
 * PrepareProposal app/prepare_proposal.go:50-53).  Construct fails on a tx
 * that does not fit or a normal tx after a blob tx; Build skips txs that do
 * not fit and returns the kept ones.
 *   txs, tx_off: the block's n_txs transactions concatenated; tx i is
 *     txs[tx_off[i] .. tx_off[i+1]) (tx_off has n_txs + 1 entries).
 *   max_square_size: appconsts.SquareSizeUpperBound / GovMaxSquareSize
 *     (power of two); threshold: appconsts.SubtreeRootThreshold (64).
 *   square_size: out, the ODS width k (dataSquare.Size()).
 *   kept (n_txs entries, may be NULL) / n_kept: indexes of the txs in the
 *     square in block order (normal txs, then blob txs) -- Build's txs result.
 * Errors: CDA_ERR_SQUARE with go-square's message (cda_last_error). */
#define CDA_SQUARE_CONSTRUCT 0
#define CDA_SQUARE_BUILD 1

/* Layout only, on the host (no device work; ctx may be NULL, then the error
 * message is cda_last_error(NULL) of the calling thread).  share_indexes
 * receives the start share of every blob, per PFB in square order and blob
 * order within the PFB (the IndexWrapper.share_indexes written to the square). */
int cda_square_layout(cda_ctx *ctx, const uint8_t *txs, const uint64_t *tx_off, uint32_t n_txs,
                      uint32_t max_square_size, uint32_t threshold, int mode, uint32_t *square_size, uint32_t *kept,
                      uint32_t *n_kept, uint32_t *share_indexes, uint32_t share_index_cap, uint32_t *n_share_indexes);

/* go-square builder.FindTxShareRange for the square.Construct layout of txs
 * (pkg/proof/proof.go:22-49 NewTxInclusionProof): the shares [start, end) of
 * the square holding kept tx tx_index (normal txs, then blob txs as their
 * IndexWrapper in the PFB namespace; *is_pfb says which).  Equal txs report
 * the last copy's range (the splitters key ranges by tx hash).  Host only;
 * ctx may be NULL.  CDA_ERR_INVALID "txIndex %u out of range". */
int cda_square_tx_share_range(cda_ctx *ctx, const uint8_t *txs, const uint64_t *tx_off, uint32_t n_txs,
                              uint32_t max_square_size, uint32_t threshold, uint32_t tx_index, uint32_t *start,
                              uint32_t *end, int *is_pfb);

/* The square's k*k shares (row-major) into ods (host, ods_capacity bytes;
 * max_square_size^2 * 512 always suffices).  Shares are written on the GPU. */
int cda_square_construct(cda_ctx *ctx, const uint8_t *txs, const uint64_t *tx_off, uint32_t n_txs,
                         uint32_t max_square_size, uint32_t threshold, int mode, uint8_t *ods, size_t ods_capacity,
                         uint32_t *square_size, uint32_t *kept, uint32_t *n_kept);

/* Construct + ExtendShares + NewDataAvailabilityHeader in one submission (the
 * proposal paths' whole DA step); the ODS never leaves HBM.  eds may be NULL;
 * row_roots / col_roots hold roots_capacity bytes each (2 * max_square_size *
 * 90 always suffices); data_root = 32 bytes. */
int cda_construct_extend_dah(cda_ctx *ctx, const uint8_t *txs, const uint64_t *tx_off, uint32_t n_txs,
                             uint32_t max_square_size, uint32_t threshold, int mode, uint8_t *eds, size_t eds_capacity,
                             uint8_t *row_roots, uint8_t *col_roots, size_t roots_capacity, uint8_t *data_root,
                             uint32_t *square_size, uint32_t *kept, uint32_t *n_kept);

/* Device variant: the layout is planned from the host txs, the shares are
 * written from d_txs (a device copy of the same bytes with >= 16 readable
 * bytes after the end) into d_ods; only enqueues on stream (NULL = HIP's
 * default stream). */
int cda_square_construct_device(cda_ctx *ctx, const uint8_t *txs, const uint64_t *tx_off, uint32_t n_txs,
                                const void *d_txs, uint32_t max_square_size, uint32_t threshold, int mode,
                                void *d_ods, size_t ods_capacity, uint32_t *square_size, uint32_t *kept,
                                uint32_t *n_kept, void *stream);

/* ---- Blob share commitments --------------------------
 * go-square v1.1.0 inclusion.CreateCommitment(blob, merkle.HashFromByteSlices,
 * threshold) for n blobs at once (x/blob/types/blob_tx.go:98 ValidateBlobTx;
 * x/blob/types/payforblob.go:53 CreateCommitments).
 *   namespaces: n * 29 bytes (version || id); blob i's data is
 *     data[data_off[i] .. data_off[i+1]) (data_off has n + 1 entries);
 *   share_versions: n bytes or NULL (all ShareVersionZero);
 *   threshold: appconsts.SubtreeRootThreshold (64);
 *   commitments: n * 32 bytes.
 * A blob with empty data commits to sha256("") (no shares).  Invalid share
 * versions / namespaces: CDA_ERR_SQUARE with go-square's message. */
int cda_blob_commitments(cda_ctx *ctx, const uint8_t *namespaces, const uint8_t *data, const uint64_t *data_off,
                         const uint8_t *share_versions, uint32_t n, uint32_t threshold, uint8_t *commitments);
/* Device variant: d_data is a device copy of the blob bytes with >= 16
 * readable bytes after the end, d_commitments is device memory; namespaces /
 * offsets / versions stay on the host (the layout is planned there).  Only
 * enqueues on stream (NULL = HIP's default stream). */
int cda_blob_commitments_device(cda_ctx *ctx, const uint8_t *namespaces, const uint64_t *data_off,
                                const uint8_t *share_versions, uint32_t n, uint32_t threshold, const void *d_data,
                                void *d_commitments, void *stream);

/* ---- Resident squares: NMT proofs and commitments from cached nodes -------
 * (SURVEY.md 8(f) row 3).  cda_square_create extends one ODS and keeps in HBM
 * the EDS, every level of every row tree (the reference's
 * EDSSubTreeRootCacher, pkg/inclusion/nmt_caching.go:80-124) and all levels
 * of the data-root tree, so proofs are index arithmetic plus one gather.
 * On CDA_ERR_PUSH_ORDER the handle is still created (the EDS exists). */
typedef struct cda_square cda_square;
int cda_square_create(cda_ctx *ctx, const uint8_t *ods, uint32_t n_shares, cda_square **out);
int cda_square_destroy(cda_square *sq);
/* Any output may be NULL: k, row/col roots (2k*90 each), data root (32), EDS ((2k)^2*512). */
int cda_square_dah(cda_square *sq, uint32_t *k, uint8_t *row_roots, uint8_t *col_roots, uint8_t *data_root,
                   uint8_t *eds);
/* proof.NewShareInclusionProofFromEDS (pkg/proof/proof.go:77-145) for the ODS
 * share range [start, end) (row-major ODS indexes), R = end_row - start_row + 1
 * rows, A = log2(4k) aunts, M = 2*log2(2k) node slots per row:
 *   shares        (end - start) * 512: ShareProof.Data, concatenated
 *   nmt_start/end R entries: NMTProof.Start / End (leaf range in the row)
 *   nmt_count     R entries; nmt_nodes R*M*90 B: NMTProof.Nodes of row i at
 *                 [i*M*90, ...) (nmt ProveRange order: maximal subtrees outside
 *                 the range, left to right); NMTProof.LeafHash is empty
 *   row_roots     R*90: RowProof.RowRoots
 *   row_leaf_hash R*32, row_aunts R*A*32: RowProof.Proofs (merkle proofs of
 *                 the rows among rowRoots || colRoots: Total 4k, Index = row,
 *                 LeafHash, Aunts bottom-up) */
int cda_square_share_proof(cda_square *sq, uint32_t start, uint32_t end, uint8_t *shares, uint32_t *start_row,
                           uint32_t *end_row, int32_t *nmt_start, int32_t *nmt_end, uint32_t *nmt_count,
                           uint8_t *nmt_nodes, uint8_t *row_roots, uint8_t *row_leaf_hash, uint8_t *row_aunts);
/* inclusion.GetCommitment (pkg/inclusion/get_commit.go:12-30) for n blobs:
 * blob i starts at ODS share starts[i] (normalised by NextShareIndex as the
 * reference does) and spans share_lens[i] shares; commitments n*32. */
int cda_square_blob_commitments(cda_square *sq, const uint32_t *starts, const uint32_t *share_lens, uint32_t n,
                                uint32_t threshold, uint8_t *commitments);
/* EDSSubTreeRootCacher.getSubTreeRoot (pkg/inclusion/nmt_caching.go:111-124):
 * the 90-B node of row tree `row` (0 <= row < 2k) reached from its root by
 * walk[0 .. walk_len) (0 = WalkLeft, 1 = WalkRight; GetCommitment prefixes
 * WalkLeft for the ODS half).  A walk longer than the tree's depth fails with
 * the cache's "did not find sub tree root: [...]" (root still receives the
 * leaf it reached); row >= 2k: "row exceeds range of cache: max %d got %d". */
int cda_square_subtree_root(cda_square *sq, uint32_t row, const uint8_t *walk, uint32_t walk_len, uint8_t *root);

/* ---- Repair ------------------------------------------
 * rsmt2d ExtendedDataSquare.Repair(rowRoots, colRoots) (EXT v0.14.0,
 * go.mod:13; used by light / full nodes after sampling).  eds: w*w*512 bytes,
 * in/out; present: w*w bytes (0 = missing: the cell's bytes are ignored and
 * reconstructed).  row_roots / col_roots: w*90 bytes each (the DAH).
 * Returns CDA_OK (eds complete), CDA_ERR_BYZANTINE (*byz_axis 0 row / 1 col,
 * *byz_index), CDA_ERR_UNREPAIRABLE, or CDA_ERR_INVALID for a complete vector
 * whose root differs from the given one ("bad root input: ..."). */
int cda_repair(cda_ctx *ctx, uint8_t *eds, const uint8_t *present, uint32_t w, const uint8_t *row_roots,
               const uint8_t *col_roots, int32_t *byz_axis, uint32_t *byz_index);
/* cda_repair on an HBM-resident square (d_eds: w*w*512 device bytes, repaired
 * in place; present and the roots stay host buffers).  Same outcomes and
 * messages; the work is ordered after everything already queued on the
 * device and complete when the call returns. */
int cda_repair_device(cda_ctx *ctx, void *d_eds, const uint8_t *present, uint32_t w, const uint8_t *row_roots,
                      const uint8_t *col_roots, int32_t *byz_axis, uint32_t *byz_index);
/* rsmt2d Codec.Decode (LeoRSCodec -> reedsolomon Reconstruct): n_codewords
 * codewords of 2*n_shards shards of shard_len bytes (multiple of 64),
 * contiguous; shards with present[] == 0 are reconstructed in place (data
 * and parity).  Fewer than n_shards present: CDA_ERR_UNREPAIRABLE. */
int cda_rs_decode(cda_ctx *ctx, uint8_t *shards, const uint8_t *present, uint32_t n_shards, uint32_t shard_len,
                  uint32_t n_codewords);

/* ---- Standalone erasured NMT trees -----------
 * wrapper.NewErasuredNamespacedMerkleTree(squareSize, axisIndex), n_cells
 * Pushes and Root() (pkg/wrapper/nmt_wrapper.go:55-124) for trees built
 * outside ComputeExtendedDataSquare (pkg/proof/proof.go:157-189,
 * pkg/inclusion/nmt_caching.go:96-109, test/util/malicious/tree.go:46-70).
 *   cells: n_trees * n_cells * cell_len bytes; push i of tree t at
 *     (t*n_cells + i)*cell_len; cell_len >= 29 (NamespaceSize).  The leaf
 *     namespace is cell[0:29] when i < square_size and axis_index[t] <
 *     square_size (isQuadrantZero, :138-140), else ParitySharesNamespace.
 *   n_cells: any count <= 2*square_size (nmt's RFC-6962 split for non powers
 *     of two); 0 gives NmtHasher.EmptyRoot.
 *   roots: n_trees * 90 bytes; status (n_trees int32, may be NULL): CDA_OK or
 *     CDA_ERR_PUSH_ORDER per tree (nmt Push ErrInvalidPushOrder; the call then
 *     returns CDA_ERR_PUSH_ORDER with the first tree's message).
 * 512-byte cells, a power-of-two n_cells and consecutive axis indexes (rows
 * of a square) run on the square kernels; anything else on generic ones. */
int cda_nmt_axis_roots(cda_ctx *ctx, const uint8_t *cells, uint32_t cell_len, uint32_t n_cells, uint32_t n_trees,
                       uint32_t square_size, const uint32_t *axis_index, uint8_t *roots, int32_t *status);
int cda_nmt_axis_root(cda_ctx *ctx, const uint8_t *cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                      uint32_t axis_index, uint8_t *root);
/* (*ErasuredNamespacedMerkleTree).ProveRange(start, end) (:126-129 -> nmt
 * ProveRange) of the tree above: nodes receives the proof nodes (90 B each, the
 * maximal subtrees outside [start, end) depth first, left to right; at most
 * 2*ceil(log2 n_cells)), *n_nodes their count, root (may be NULL) the root.
 * start >= end or end > n_cells: CDA_ERR_INVALID ("invalid proof range"). */
int cda_nmt_prove_range(cda_ctx *ctx, const uint8_t *cells, uint32_t cell_len, uint32_t n_cells, uint32_t square_size,
                        uint32_t axis_index, uint32_t start, uint32_t end, uint8_t *nodes, uint32_t *n_nodes,
                        uint8_t *root);
/* go-square/merkle HashFromByteSlices (RFC-6962) over n byte slices, item i =
 * items[off[i] .. off[i+1]) (off has n + 1 entries): (*DataAvailabilityHeader)
 * .Hash for any root count and size (data_availability_header.go:92-108).
 * n == 0 gives sha256(""). */
int cda_merkle_root(cda_ctx *ctx, const uint8_t *items, const uint64_t *off, uint32_t n, uint8_t out[32]);

/* Stage timing (HIP events on the launch stream).  When enabled, every
 * enqueued stage is bracketed by events; cda_stage_times synchronises them and
 * returns, per stage, the summed milliseconds and launch counts since the
 * previous call, then resets.  Stages: 0 RS Q0 (rows+cols), 1 RS Q3, 2 push-
 * order check, 3 NMT leaves, 4 NMT levels, 5 data root. */
#define CDA_NUM_STAGES 6
int cda_set_profiling(cda_ctx *ctx, int enable);
int cda_stage_times(cda_ctx *ctx, double *ms, uint32_t *counts, int n_stages);

#ifdef __cplusplus
}
#endif

#endif /* CDA_H */
