// comm.cpp -- the multi-GPU boundary of the path (SURVEY.md 8b "eegfx_gather", 8e).
//
// After host marker planning every selected epoch is independent (OffLineDataProvider.java:
// 200-265 is the only sequential state), so ranks take contiguous ranges of the selected-epoch
// list and run the fused kernels on their range with no collective.  The one exchange is
// assembling the per-rank feature rows in rank order -- the reference's getData() list order --
// which eegfx_gather does with one RCCL broadcast per rank inside a group: shards may differ by a
// row (eegfx_shard_range), and a rooted broadcast writes each shard straight into its final rows
// of `out` with no padding or compaction pass.  RCCL runs over xGMI (peer-to-peer links) on an
// MI355X node.  Normalisation is per row, so there is no statistic to all-reduce.
// eegfx_gather_root assembles the matrix on one rank only (the reference's single consumer):
// grouped ncclSend / ncclRecv, every shard crossing one xGMI link once.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "common.h"

using namespace eegfx;

struct eegfx_comm {
  ncclComm_t comm = nullptr;
  eegfx_ctx* ctx = nullptr;
  int world = 1, rank = 0;
};

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) fail(EEGFX_EHIP, "%s: %s", what, ncclGetErrorString(r));
}

void shard(int64_t n, int world, int rank, int64_t* s, int64_t* e) {
  const int64_t base = n / world, extra = n % world;
  *s = rank * base + (rank < extra ? rank : extra);
  *e = *s + base + (rank < extra ? 1 : 0);
}

}  // namespace

extern "C" {

int eegfx_shard_range(int64_t n, int32_t rank, int32_t world, int64_t* start, int64_t* end) {
  return guarded([&] {
    if (n < 0 || world < 1 || rank < 0 || rank >= world || !start || !end)
      fail(EEGFX_EINVAL, "shard_range(n=%lld, rank=%d, world=%d)", (long long)n, rank, world);
    shard(n, world, rank, start, end);
  });
}

int eegfx_gather_schedule(int64_t n_total, int32_t world, int64_t* offsets, int64_t* counts) {
  return guarded([&] {
    if (n_total < 0 || world < 1 || !offsets || !counts)
      fail(EEGFX_EINVAL, "gather_schedule(n=%lld, world=%d)", (long long)n_total, world);
    for (int r = 0; r < world; ++r) {
      int64_t s = 0, e = 0;
      shard(n_total, world, r, &s, &e);
      offsets[r] = s;
      counts[r] = e - s;
    }
  });
}

int eegfx_comm_unique_id(void* id) {
  return guarded([&] {
    if (!id) fail(EEGFX_EINVAL, "null id buffer");
    static_assert(sizeof(ncclUniqueId) == EEGFX_COMM_ID_BYTES, "unique id size");
    nccl_check(ncclGetUniqueId((ncclUniqueId*)id), "ncclGetUniqueId");
  });
}

int eegfx_comm_create(eegfx_ctx* ctx, int32_t world, int32_t rank, const void* id,
                      eegfx_comm** out) {
  return guarded([&] {
    if (!ctx || !id || !out) fail(EEGFX_EINVAL, "null argument");
    if (world < 1 || rank < 0 || rank >= world) fail(EEGFX_EINVAL, "rank %d of %d", rank, world);
    *out = nullptr;
    auto* c = new eegfx_comm;
    c->ctx = ctx;
    c->world = world;
    c->rank = rank;
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) {
      delete c;
      fail(EEGFX_EHIP, "hipSetDevice(%d)", ctx_device(ctx));
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
    if (r != ncclSuccess) {
      delete c;
      nccl_check(r, "ncclCommInitRank");
    }
    *out = c;
  });
}

int eegfx_comm_init_all(eegfx_ctx* const* ctxs, int32_t n, eegfx_comm** out) {
  return guarded([&] {
    if (!ctxs || !out || n < 1) fail(EEGFX_EINVAL, "init_all: %d contexts", n);
    std::vector<int> dev((size_t)n);
    for (int i = 0; i < n; ++i) {
      if (!ctxs[i]) fail(EEGFX_EINVAL, "null context %d", i);
      dev[(size_t)i] = ctx_device(ctxs[i]);
      out[i] = nullptr;
    }
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    nccl_check(ncclCommInitAll(comms.data(), n, dev.data()), "ncclCommInitAll");
    for (int i = 0; i < n; ++i) {
      auto* c = new eegfx_comm;
      c->comm = comms[(size_t)i];
      c->ctx = ctxs[i];
      c->world = n;
      c->rank = i;
      out[i] = c;
    }
  });
}

int eegfx_comm_rank(const eegfx_comm* comm, int32_t* rank, int32_t* world) {
  return guarded([&] {
    if (!comm || !rank || !world) fail(EEGFX_EINVAL, "null argument");
    *rank = comm->rank;
    *world = comm->world;
  });
}

int eegfx_gather(eegfx_comm* comm, const double* local, int64_t n_total, int64_t cols,
                 double* out) {
  return guarded([&] {
    if (!comm || !out || n_total < 0 || cols < 1) fail(EEGFX_EINVAL, "gather arguments");
    std::vector<int64_t> off((size_t)comm->world), cnt((size_t)comm->world);
    const int rc = eegfx_gather_schedule(n_total, comm->world, off.data(), cnt.data());
    if (rc != EEGFX_OK) fail(rc, "%s", last_error().c_str());
    if (cnt[(size_t)comm->rank] > 0 && !local) fail(EEGFX_EINVAL, "null local rows");
    if (hipSetDevice(ctx_device(comm->ctx)) != hipSuccess)
      fail(EEGFX_EHIP, "hipSetDevice(%d)", ctx_device(comm->ctx));
    const hipStream_t st = (hipStream_t)ctx_stream(comm->ctx);
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    ncclResult_t r = ncclSuccess;
    for (int root = 0; root < comm->world && r == ncclSuccess; ++root) {
      if (cnt[(size_t)root] == 0) continue;  // same decision on every rank
      r = ncclBroadcast(root == comm->rank ? (const void*)local : nullptr,
                        out + off[(size_t)root] * cols, (size_t)(cnt[(size_t)root] * cols),
                        ncclDouble, root, comm->comm, st);
    }
    const ncclResult_t g = ncclGroupEnd();
    nccl_check(r, "ncclBroadcast");
    nccl_check(g, "ncclGroupEnd");
  });
}

int eegfx_gather_root_plan(int64_t n_total, int32_t world, int32_t rank, int32_t root,
                           eegfx_gather_op* ops, int32_t* n_ops) {
  return guarded([&] {
    if (n_total < 0 || world < 1 || rank < 0 || rank >= world || root < 0 || root >= world ||
        !ops || !n_ops)
      fail(EEGFX_EINVAL, "gather_root_plan(n=%lld, world=%d, rank=%d, root=%d)",
           (long long)n_total, world, rank, root);
    int k = 0;
    for (int r = 0; r < world; ++r) {
      int64_t s = 0, e = 0;
      shard(n_total, world, r, &s, &e);
      if (e == s) continue;  // a rank without rows takes part in nothing
      if (rank == root) {
        ops[k++] = eegfx_gather_op{r == root ? EEGFX_GATHER_COPY : EEGFX_GATHER_RECV, r, s, e - s};
      } else if (r == rank) {
        ops[k++] = eegfx_gather_op{EEGFX_GATHER_SEND, root, s, e - s};
      }
    }
    *n_ops = k;
  });
}

int eegfx_gather_root(eegfx_comm* comm, const double* local, int64_t n_total, int64_t cols,
                      int32_t root, double* out) {
  return guarded([&] {
    if (!comm || n_total < 0 || cols < 1) fail(EEGFX_EINVAL, "gather_root arguments");
    if (root < 0 || root >= comm->world) fail(EEGFX_EINVAL, "root %d of %d", root, comm->world);
    std::vector<eegfx_gather_op> ops((size_t)comm->world);
    int32_t k = 0;
    const int rc = eegfx_gather_root_plan(n_total, comm->world, comm->rank, root, ops.data(), &k);
    if (rc != EEGFX_OK) fail(rc, "%s", last_error().c_str());
    if (comm->rank == root && n_total > 0 && !out) fail(EEGFX_EINVAL, "null out on the root");
    for (int i = 0; i < k; ++i)
      if (ops[(size_t)i].kind != EEGFX_GATHER_RECV && !local) fail(EEGFX_EINVAL, "null local rows");
    if (hipSetDevice(ctx_device(comm->ctx)) != hipSuccess)
      fail(EEGFX_EHIP, "hipSetDevice(%d)", ctx_device(comm->ctx));
    const hipStream_t st = (hipStream_t)ctx_stream(comm->ctx);
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    ncclResult_t r = ncclSuccess;
    hipError_t h = hipSuccess;
    for (int i = 0; i < k && r == ncclSuccess && h == hipSuccess; ++i) {
      const eegfx_gather_op& op = ops[(size_t)i];
      const size_t count = (size_t)(op.rows * cols);
      if (op.kind == EEGFX_GATHER_SEND) {
        r = ncclSend(local, count, ncclDouble, op.peer, comm->comm, st);
      } else if (op.kind == EEGFX_GATHER_RECV) {
        r = ncclRecv(out + op.row * cols, count, ncclDouble, op.peer, comm->comm, st);
      } else if (local != out + op.row * cols) {  // the root's own rows
        h = hipMemcpyAsync(out + op.row * cols, local, sizeof(double) * count,
                           hipMemcpyDeviceToDevice, st);
      }
    }
    const ncclResult_t g = ncclGroupEnd();
    nccl_check(r, "ncclSend/ncclRecv");
    if (h != hipSuccess) fail(EEGFX_EHIP, "hipMemcpyAsync: %s", hipGetErrorString(h));
    nccl_check(g, "ncclGroupEnd");
  });
}

int eegfx_group_start(void) {
  return guarded([&] { nccl_check(ncclGroupStart(), "ncclGroupStart"); });
}

int eegfx_group_end(void) {
  return guarded([&] { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); });
}

int eegfx_comm_destroy(eegfx_comm* comm) {
  return guarded([&] {
    if (!comm) return;
    const ncclResult_t r = comm->comm ? ncclCommDestroy(comm->comm) : ncclSuccess;
    delete comm;
    nccl_check(r, "ncclCommDestroy");
  });
}

}  // extern "C"
