// comm.hip — the sequence-shard collectives of include/rtkv.h on RCCL (host code, no kernels).
//
// The shard driver (include/rtkv.h "Sequence shards") has two data exchanges per layer:
//   step 2  all-gather of A (4 B per token)                   rtkv_allgather_rows
//   end     every rank's packed K/V byte ranges + scale/zp    rtkv_allgather_packed
// Both are grouped point-to-point launches of exact byte ranges (no padding to the largest rank), the
// pattern rtkv/sharded.py issues through torch.distributed; here a host in any language drives them
// through the C ABI with its own communicator (rtkv_comm_unique_id / rtkv_comm_init).
//
// RCCL is resolved at first use with dlopen("librccl.so.1"): librtkv.so has no link-time RCCL
// dependency, and a process that already loaded an RCCL (PyTorch's, same soname) shares that copy.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "common.h"

namespace rtkv {
namespace {

struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        r.why = std::string("RCCL lacks ") + name;
      }
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.init_rank, "ncclCommInitRank");
    sym(r.destroy, "ncclCommDestroy");
    sym(r.count, "ncclCommCount");
    sym(r.user_rank, "ncclCommUserRank");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.error_string, "ncclGetErrorString");
    r.ok = all;
  });
  return r;
}

#define RTKV_RCCL(expr)                                                                          \
  do {                                                                                           \
    const ncclResult_t _r = (expr);                                                              \
    if (_r != ncclSuccess) {                                                                     \
      ::rtkv::set_error(std::string(#expr) + ": " + rccl().error_string(_r));                    \
      return RTKV_ERR_HIP;                                                                       \
    }                                                                                            \
  } while (0)

int need_rccl() {
  if (!rccl().ok) {
    set_error("rtkv comm: " + rccl().why);
    return RTKV_ERR_UNSUPPORTED;
  }
  return RTKV_OK;
}

// Inside a group: remember the first failing send/recv and keep going, so that the group is always
// closed (an RCCL group left open on this thread would capture every later RCCL call of the thread).
struct GroupErr {
  ncclResult_t r = ncclSuccess;
  const char* what = nullptr;
  void note(ncclResult_t x, const char* w) {
    if (x != ncclSuccess && r == ncclSuccess) { r = x; what = w; }
  }
  int close() {  // ncclGroupEnd, then the first error of the group or of the end itself
    const ncclResult_t e = rccl().group_end();
    if (r != ncclSuccess) {
      set_error(std::string(what) + ": " + rccl().error_string(r));
      return RTKV_ERR_HIP;
    }
    if (e != ncclSuccess) {
      set_error(std::string("ncclGroupEnd: ") + rccl().error_string(e));
      return RTKV_ERR_HIP;
    }
    return RTKV_OK;
  }
};

int comm_shape(ncclComm_t c, int* rank, int* nranks) {
  RTKV_RCCL(rccl().user_rank(c, rank));
  RTKV_RCCL(rccl().count(c, nranks));
  return RTKV_OK;
}

}  // namespace
}  // namespace rtkv

using namespace rtkv;

extern "C" {

int rtkv_comm_unique_id(uint8_t* id, size_t id_bytes) {
  if (int rc = need_rccl()) return rc;
  RTKV_REQUIRE(id && id_bytes >= sizeof(ncclUniqueId), "rtkv_comm_unique_id: id buffer < RTKV_COMM_ID_BYTES");
  ncclUniqueId u;
  RTKV_RCCL(rccl().get_unique_id(&u));
  std::memcpy(id, u.internal, sizeof(u.internal));
  return RTKV_OK;
}

int rtkv_comm_init(void** comm, const uint8_t* id, size_t id_bytes, int32_t nranks, int32_t rank) {
  if (int rc = need_rccl()) return rc;
  RTKV_REQUIRE(comm && id && id_bytes >= sizeof(ncclUniqueId), "rtkv_comm_init: bad arguments");
  RTKV_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "rtkv_comm_init: rank out of range");
  ncclUniqueId u;
  std::memcpy(u.internal, id, sizeof(u.internal));
  ncclComm_t c = nullptr;
  RTKV_RCCL(rccl().init_rank(&c, nranks, u, rank));
  *comm = c;
  return RTKV_OK;
}

int rtkv_comm_destroy(void* comm) {
  if (!comm) return RTKV_OK;
  if (int rc = need_rccl()) return rc;
  RTKV_RCCL(rccl().destroy(static_cast<ncclComm_t>(comm)));
  return RTKV_OK;
}

int rtkv_allgather_rows(void* comm, const float* a_local_dev, float* a_dev, int64_t B, int64_t S_local,
                        void* stream) {
  if (int rc = need_rccl()) return rc;
  RTKV_REQUIRE(comm && a_local_dev && a_dev && B >= 1 && S_local >= 1, "rtkv_allgather_rows: bad arguments");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int me, n;
  if (int rc = comm_shape(c, &me, &n)) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t S_total = S_local * n;
  // own rows: a device copy into their global position (batch row b: [b][me*S_local, +S_local))
  RTKV_HIP_CHECK(hipMemcpy2DAsync(a_dev + (int64_t)me * S_local, (size_t)S_total * 4, a_local_dev,
                                  (size_t)S_local * 4, (size_t)S_local * 4, (size_t)B, hipMemcpyDeviceToDevice, st));
  if (n == 1) return RTKV_OK;
  RTKV_RCCL(rccl().group_start());
  GroupErr ge;
  for (int64_t b = 0; b < B; ++b)
    for (int j = 0; j < n; ++j) {
      if (j == me) continue;
      ge.note(rccl().send(a_local_dev + b * S_local, (size_t)S_local, ncclFloat32, j, c, st), "ncclSend");
      ge.note(rccl().recv(a_dev + b * S_total + (int64_t)j * S_local, (size_t)S_local, ncclFloat32, j, c, st),
              "ncclRecv");
    }
  return ge.close();
}

int rtkv_allgather_packed(void* comm, const int64_t* ranges_host, int64_t B, int64_t row_capacity,
                          const rtkv_layer_out* out, void* stream) {
  if (int rc = need_rccl()) return rc;
  RTKV_REQUIRE(comm && ranges_host && out && B >= 1 && row_capacity >= 1, "rtkv_allgather_packed: bad arguments");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int me, n;
  if (int rc = comm_shape(c, &me, &n)) return rc;
  if (n == 1) return RTKV_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // ranges_host[(b*(n+1) + j)*2 + {0,1}] = {first row, first packed byte} of rank j in batch row b
  auto row = [&](int64_t b, int j) { return ranges_host[(b * (n + 1) + j) * 2]; };
  auto byte = [&](int64_t b, int j) { return ranges_host[(b * (n + 1) + j) * 2 + 1]; };
  for (int64_t b = 0; b < B; ++b)
    for (int j = 0; j < n; ++j)
      RTKV_REQUIRE(row(b, j) <= row(b, j + 1) && row(b, n) <= row_capacity && byte(b, j) <= byte(b, j + 1) &&
                       (!out->packed_k_dev || byte(b, n) <= out->packed_capacity),
                   "rtkv_allgather_packed: ranges not ascending or beyond the buffers");
  RTKV_RCCL(rccl().group_start());
  GroupErr ge;
  for (int64_t b = 0; b < B; ++b)
    for (int j = 0; j < n; ++j) {
      if (j == me) continue;
      // the same three spans of rank `src` travel from src to everyone else
      for (int dir = 0; dir < 2; ++dir) {
        const int src = dir == 0 ? me : j;
        const int64_t b0 = byte(b, src), b1 = byte(b, src + 1);
        const int64_t r0 = row(b, src), r1 = row(b, src + 1);
        auto xfer = [&](void* base, int64_t lo, int64_t hi, ncclDataType_t t) -> ncclResult_t {
          if (!base || hi <= lo) return ncclSuccess;
          const size_t esz = t == ncclFloat32 ? 4 : 1;
          char* p = static_cast<char*>(base) + lo * (int64_t)esz;
          return dir == 0 ? rccl().send(p, (size_t)(hi - lo), t, j, c, st) : rccl().recv(p, (size_t)(hi - lo), t, j, c, st);
        };
        const char* op = dir == 0 ? "ncclSend" : "ncclRecv";
        ge.note(xfer(out->packed_k_dev, b0, b1, ncclUint8), op);
        ge.note(xfer(out->packed_v_dev, b0, b1, ncclUint8), op);
        ge.note(xfer(out->scale_zp_dev, (b * row_capacity + r0) * 4, (b * row_capacity + r1) * 4, ncclFloat32), op);
      }
    }
  return ge.close();
}

}  // extern "C"
