// Frame-parallel result gather over RCCL (SURVEY §8e, §5 "failure detection").
//
// Frames shard round-robin over one process per GPU (frame i -> rank i % world; __call__ keeps no
// cross-frame state, pose_detector.py:484-517), so the data path has no collective.  The only
// exchange is the per-frame result records, gathered to rank 0 straight from device memory:
//
//   compute stream:  ... post-process of step k -> pack_records (runtime.hip) -> ev_packed[slot]
//   comm stream:     wait ev_packed[slot] -> ncclGather(records -> root) -> D2H (root, pinned)
//                    -> ev_done[slot]
//
// Two record slots, so step k's gather overlaps step k+1's forward; op_comm_wait() takes the
// oldest outstanding gather and gives up after a per-rank timeout (a stalled or dead rank): it
// aborts the communicator (ncclCommAbort) and returns OP_ERR_TIMEOUT instead of hanging.
// The communicator is created non-blocking (ncclConfig_t.blocking = 0) so initialisation obeys the
// same timeout.  Host code passes RCCL's 128-byte unique id between ranks (frames.py: TCP).
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "common.hpp"

extern "C" int64_t record_bytes(int max_persons);
extern "C" int ctx_pack_records(op_ctx* c, int first, int n, int max_persons, int64_t frame_base, int frame_stride,
                                void* dst, hipStream_t* stream, int keep_slot);
extern "C" int ctx_kept_overflow(op_ctx* c, int slot, int32_t* frames, int32_t* reasons, int32_t cap, int32_t* count);
extern "C" int ctx_kept_result(op_ctx* c, int slot, int frame, double* poses, double* scores, int32_t cap,
                               op_frame_result* res);
extern "C" int ctx_device(op_ctx* c);

struct op_comm {
  ncclComm_t comm = nullptr;
  int world = 0, rank = 0, device = 0;
  hipStream_t stream = nullptr;
  char* d_rec[2] = {nullptr, nullptr};  // this rank's records of one step
  char* d_all[2] = {nullptr, nullptr};  // root: every rank's records
  char* h_all[2] = {nullptr, nullptr};  // root: pinned host copy
  size_t rec_cap = 0, all_cap = 0;      // bytes per slot
  hipEvent_t ev_packed[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  int next = 0;                         // slot of the next submit
  int queued[2] = {0, 0};               // frames (all ranks) of an outstanding gather per slot, 0 = none
  int64_t rbytes[2] = {0, 0};
  int last = -1;                        // slot op_comm_wait returned last (op_comm_overflow*)
  int order[2] = {-1, -1};              // FIFO of outstanding slots
  bool aborted = false;
  double timeout_s = 0.0;               // op_comm_create's per-rank timeout (init and enqueue waits)
};

namespace {

using op::set_error;

#define RC(x)            \
  do {                   \
    int _rc = (x);       \
    if (_rc) return _rc; \
  } while (0)

int nccl_fail(const char* what, ncclResult_t r) {
  set_error(std::string(what) + ": " + ncclGetErrorString(r));
  return OP_ERR_HIP;
}

// Poll `ready` until it returns true, the communicator reports an asynchronous error, or the timeout
// expires (then abort the communicator so no RCCL kernel is left waiting on a peer).
template <class F>
int wait_for(op_comm* g, double timeout_s, const char* what, F ready) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int r = ready();
    if (r == 1) return OP_OK;
    if (r < 0) return OP_ERR_HIP;
    ncclResult_t ae = ncclSuccess;
    if (g->comm && ncclCommGetAsyncError(g->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      (void)ncclCommAbort(g->comm);
      g->comm = nullptr;
      g->aborted = true;
      return nccl_fail(what, ae);
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s) {
      if (g->comm) (void)ncclCommAbort(g->comm);
      g->comm = nullptr;
      g->aborted = true;
      set_error(std::string(what) + ": timed out after " + std::to_string(timeout_s) +
                " s (a rank stalled or died); communicator aborted");
      return OP_ERR_TIMEOUT;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int grow(char** p, size_t* cap, size_t bytes, bool host) {
  if (bytes <= *cap) return OP_OK;
  if (*p) {
    if (host) OP_HIP_CHECK(hipHostFree(*p));
    else OP_HIP_CHECK(hipFree(*p));
  }
  *p = nullptr;
  if (host) OP_HIP_CHECK(hipHostMalloc((void**)p, bytes, hipHostMallocDefault));
  else OP_HIP_CHECK(hipMalloc((void**)p, bytes));
  return OP_OK;
}

}  // namespace

extern "C" {

int op_comm_unique_id(uint8_t* id) {
  if (!id) return OP_ERR_INVALID;
  static_assert(sizeof(ncclUniqueId) == OP_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
  memcpy(id, &u, sizeof(u));
  return OP_OK;
}

int op_comm_create(op_ctx* ctx, int32_t world, int32_t rank, const uint8_t* id, double timeout_s, op_comm** out) {
  if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world || timeout_s <= 0) {
    set_error("op_comm_create: bad arguments");
    return OP_ERR_INVALID;
  }
  *out = nullptr;
  op_comm* g = new op_comm();
  g->world = world;
  g->rank = rank;
  g->device = ctx_device(ctx);
  g->timeout_s = timeout_s;
  auto fail = [&](int rc) {
    if (g->comm) (void)ncclCommAbort(g->comm);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
    return rc;
  };
  if (hipSetDevice(g->device) != hipSuccess || hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    set_error("op_comm_create: stream");
    return fail(OP_ERR_HIP);
  }
  for (int k = 0; k < 2; ++k) {
    if (hipEventCreateWithFlags(&g->ev_packed[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_done[k], hipEventDisableTiming) != hipSuccess) {
      set_error("op_comm_create: events");
      return fail(OP_ERR_HIP);
    }
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // initialisation and collectives return at once; op_comm_wait polls with a timeout
  ncclResult_t r = ncclCommInitRankConfig(&g->comm, world, u, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    g->comm = nullptr;
    return fail(nccl_fail("ncclCommInitRankConfig", r));
  }
  int rc = wait_for(g, timeout_s, "RCCL communicator init", [&]() -> int {
    ncclResult_t ae = ncclInProgress;
    if (ncclCommGetAsyncError(g->comm, &ae) != ncclSuccess) return -1;
    return ae == ncclSuccess ? 1 : 0;
  });
  if (rc) return fail(rc);
  *out = g;
  return OP_OK;
}

int op_comm_destroy(op_comm* g) {
  if (!g) return OP_OK;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  if (g->comm) {
    if (g->aborted) (void)ncclCommAbort(g->comm);
    else (void)ncclCommDestroy(g->comm);
  }
  for (int k = 0; k < 2; ++k) {
    if (g->d_rec[k]) (void)hipFree(g->d_rec[k]);
    if (g->d_all[k]) (void)hipFree(g->d_all[k]);
    if (g->h_all[k]) (void)hipHostFree(g->h_all[k]);
    if (g->ev_packed[k]) (void)hipEventDestroy(g->ev_packed[k]);
    if (g->ev_done[k]) (void)hipEventDestroy(g->ev_done[k]);
  }
  if (g->stream) (void)hipStreamDestroy(g->stream);
  delete g;
  return OP_OK;
}

int op_comm_gather_results(op_comm* g, op_ctx* ctx, int32_t first, int32_t n, int32_t max_persons, int64_t frame_base,
                           int32_t frame_stride) {
  if (!g || !ctx || n < 1 || max_persons < 0) {
    set_error("op_comm_gather_results: bad arguments");
    return OP_ERR_INVALID;
  }
  if (!g->comm) {
    set_error("op_comm_gather_results: communicator aborted");
    return OP_ERR_STATE;
  }
  const int k = g->next;
  if (g->queued[k]) {
    set_error("op_comm_gather_results: two gathers outstanding; op_comm_wait first");
    return OP_ERR_STATE;
  }
  OP_HIP_CHECK(hipSetDevice(g->device));
  const int64_t rb = record_bytes(max_persons);
  const size_t mine = (size_t)n * rb, all = mine * g->world;
  if (mine > g->rec_cap || (g->rank == 0 && all > g->all_cap)) {  // grow every slot at once
    if (g->order[0] >= 0) {
      set_error("op_comm_gather_results: record size grew with a gather outstanding; op_comm_wait first");
      return OP_ERR_STATE;
    }
    OP_HIP_CHECK(hipStreamSynchronize(g->stream));
    for (int s = 0; s < 2; ++s) {
      size_t c = g->rec_cap;
      RC(grow(&g->d_rec[s], &c, mine, false));
      if (g->rank == 0) {
        c = g->all_cap;
        RC(grow(&g->d_all[s], &c, all, false));
        c = g->all_cap;
        RC(grow(&g->h_all[s], &c, all, true));
      }
    }
    g->rec_cap = std::max(g->rec_cap, mine);
    if (g->rank == 0) g->all_cap = std::max(g->all_cap, all);
  }
  // packing rewrites slot k's keep buffers (overflow headers, rows, maps): a waited-for gather in
  // that slot can no longer be queried (op_comm_overflow* then report OP_ERR_STATE, never a mix of
  // two steps' data)
  if (g->last == k) g->last = -1;
  hipStream_t cst;
  RC(ctx_pack_records(ctx, first, n, max_persons, frame_base, frame_stride, g->d_rec[k], &cst, k));
  OP_HIP_CHECK(hipEventRecord(g->ev_packed[k], cst));
  OP_HIP_CHECK(hipStreamWaitEvent(g->stream, g->ev_packed[k], 0));
  // one rank: the gather is the identity, so the root's D2H copy reads the packed records directly
  // (round 6: the one-rank ncclGather ran as an 11-us copy kernel per step)
  const bool alone = g->world == 1;
  ncclResult_t r = alone ? ncclSuccess
                         : ncclGather(g->d_rec[k], g->rank == 0 ? g->d_all[k] : nullptr, mine, ncclUint8, 0, g->comm,
                                      g->stream);
  if (r != ncclSuccess && r != ncclInProgress) return nccl_fail("ncclGather", r);
  if (r == ncclInProgress) {
    // non-blocking communicator: the gather may still be on its way into g->stream; the root's D2H
    // copy must be enqueued behind it, so wait until RCCL reports the call complete (bounded)
    RC(wait_for(g, g->timeout_s, "ncclGather enqueue", [&]() -> int {
      ncclResult_t ae = ncclInProgress;
      if (ncclCommGetAsyncError(g->comm, &ae) != ncclSuccess) return -1;
      return ae == ncclSuccess ? 1 : 0;  // an error state is reported (and aborted) by wait_for
    }));
  }
  if (g->rank == 0)
    OP_HIP_CHECK(hipMemcpyAsync(g->h_all[k], alone ? g->d_rec[k] : g->d_all[k], all, hipMemcpyDeviceToHost, g->stream));
  OP_HIP_CHECK(hipEventRecord(g->ev_done[k], g->stream));
  g->queued[k] = n * g->world;
  g->rbytes[k] = rb;
  if (g->order[0] < 0) g->order[0] = k;
  else g->order[1] = k;
  g->next = k ^ 1;
  return OP_OK;
}

int op_comm_wait(op_comm* g, double timeout_s, const void** records, int32_t* n_frames, int64_t* rec_bytes) {
  if (!g || !records || !n_frames || !rec_bytes || timeout_s <= 0) {
    set_error("op_comm_wait: bad arguments");
    return OP_ERR_INVALID;
  }
  const int k = g->order[0];
  if (k < 0) {
    set_error("op_comm_wait: no gather outstanding");
    return OP_ERR_STATE;
  }
  OP_HIP_CHECK(hipSetDevice(g->device));
  int rc = wait_for(g, timeout_s, "RCCL result gather", [&]() -> int {
    hipError_t e = hipEventQuery(g->ev_done[k]);
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    set_error(std::string("hipEventQuery: ") + hipGetErrorString(e));
    return -1;
  });
  g->order[0] = g->order[1];
  g->order[1] = -1;
  const int nf = g->queued[k];
  g->queued[k] = 0;
  if (rc) return rc;
  g->last = k;
  *records = g->rank == 0 ? g->h_all[k] : nullptr;
  *n_frames = g->rank == 0 ? nf : 0;
  *rec_bytes = g->rbytes[k];
  return OP_OK;
}

int op_comm_overflow(op_comm* g, op_ctx* ctx, int32_t* frames, int32_t* reasons, int32_t cap, int32_t* count) {
  if (!g || !ctx || !count) {
    set_error("op_comm_overflow: bad arguments");
    return OP_ERR_INVALID;
  }
  if (g->last < 0) {
    set_error("op_comm_overflow: no gather waited for yet");
    return OP_ERR_STATE;
  }
  return ctx_kept_overflow(ctx, g->last, frames, reasons, cap, count);
}

int op_comm_overflow_result(op_comm* g, op_ctx* ctx, int32_t frame, double* poses, double* scores, int32_t cap,
                            op_frame_result* res) {
  if (!g || !ctx) {
    set_error("op_comm_overflow_result: bad arguments");
    return OP_ERR_INVALID;
  }
  if (g->last < 0) {
    set_error("op_comm_overflow_result: no gather waited for yet");
    return OP_ERR_STATE;
  }
  OP_HIP_CHECK(hipSetDevice(g->device));
  return ctx_kept_result(ctx, g->last, frame, poses, scores, cap, res);
}

}  // extern "C"
