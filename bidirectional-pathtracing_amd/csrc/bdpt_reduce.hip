// bdpt_reduce.hip — the multi-GPU frame reduce of the C-ABI (bdpt_reduce_*, ABI v9).
//
// Why a whole-frame sum: the t = 1 light-tracing splats of a sample land on any pixel
// (bidirection.cpp:457-466), so GPUs that split the sample range of every pixel each hold a full
// W x H x 3 partial frame, and the image is their sum (the reference instead runs
// N CPU threads on one shared frame, raytraced_renderer.cpp:325-327).
//
// How: one RCCL communicator clique over the distinct devices of the contexts (ncclCommInitAll,
// once, at bdpt_reduce_create), then per bdpt_reduce_frames one grouped ncclReduce (sum, fp32) of
// the eye frame and one of the light frame of each device into the root context's frames, each on
// that device's stream, over xGMI. Contexts that share a device (e.g. --devices 0,0 on a one-GPU
// box) are first summed on that device by k_frame_acc into a per-device scratch pair, since RCCL
// refuses two ranks on one GPU. Under the PathTracer the sampleCountBuffer is reduced the same way
// (int32), so the root then holds every pixel's count as well.
//
// RCCL is loaded with dlopen (RTLD_LOCAL) on first use: a process that never reduces does not
// map it, and a torch process's own bundled RCCL (no SONAME) is not interposed. No fallback: if
// RCCL cannot be loaded or a call fails, the entry point fails with BDPT_E_DEVICE and the text.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bdpt_ctx.h"

using bdpt::Ctx;
using bdpt::g_err;

namespace {

struct Rccl {
  void* h = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclReduce) Reduce = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclGetVersion) GetVersion = nullptr;
  std::string err;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.h) break;
    }
    if (!r.h) { r.err = std::string("cannot load RCCL (librccl.so.1): ") + dlerror(); return; }
    auto sym = [](void* h, const char* s) { return dlsym(h, s); };
    r.CommInitAll = (decltype(r.CommInitAll))sym(r.h, "ncclCommInitAll");
    r.CommDestroy = (decltype(r.CommDestroy))sym(r.h, "ncclCommDestroy");
    r.Reduce = (decltype(r.Reduce))sym(r.h, "ncclReduce");
    r.GroupStart = (decltype(r.GroupStart))sym(r.h, "ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym(r.h, "ncclGroupEnd");
    r.GetErrorString = (decltype(r.GetErrorString))sym(r.h, "ncclGetErrorString");
    r.GetVersion = (decltype(r.GetVersion))sym(r.h, "ncclGetVersion");
    if (!r.CommInitAll || !r.CommDestroy || !r.Reduce || !r.GroupStart || !r.GroupEnd || !r.GetErrorString ||
        !r.GetVersion)
      r.err = "RCCL is missing an entry point (ncclCommInitAll / ncclReduce / ncclGroupStart ...)";
  });
  return r;
}

#define NCCLCHK(x)                                                                       \
  do {                                                                                   \
    ncclResult_t e_ = (x);                                                               \
    if (e_ != ncclSuccess) {                                                             \
      g_err = std::string("RCCL ") + #x + ": " + rccl().GetErrorString(e_);              \
      return BDPT_E_DEVICE;                                                              \
    }                                                                                    \
  } while (0)

// dst (+)= src over n floats, 16 B per lane (frames are W*H*3 floats from hipMalloc: 256-B
// aligned; the tail of n % 4 is done by the first lanes). HBM-bound streaming: one read of src (and
// of dst when accumulating), one write of dst.
__global__ void k_frame_acc(float* __restrict__ dst, const float* __restrict__ src, long long n, int accumulate) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 s = ((const float4*)src)[i];
    if (accumulate) {
      const float4 d = ((const float4*)dst)[i];
      s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
    }
    ((float4*)dst)[i] = s;
  }
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (n & 3)) {
    const long long k = (n4 << 2) + t;
    dst[k] = accumulate ? dst[k] + src[k] : src[k];
  }
}

__global__ void k_count_acc(int* __restrict__ dst, const int* __restrict__ src, long long n, int accumulate) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = accumulate ? dst[i] + src[i] : src[i];
}

}  // namespace

// One RCCL rank per distinct device.
struct bdpt_reducer {
  std::vector<Ctx*> ctxs;
  std::vector<int> rank_of;                 // ctx index -> rank (its device's)
  std::vector<int> devs;                    // rank -> device
  std::vector<std::vector<int>> members;    // rank -> ctx indices on that device
  std::vector<ncclComm_t> comms;            // rank -> communicator
  // rank -> scratch (eye | light | counts) for devices holding more than one ctx
  std::vector<float*> scratch;
  std::vector<hipEvent_t> ev;               // ctx index -> ordering event
  std::vector<int> ctx_dev;                 // ctx index -> device (the reducer's own copy)
  std::vector<hipEvent_t> done;             // rank -> recorded after its last reduce on its lead stream
  size_t npix = 0;
  bool pt = false;
};

namespace {

void free_reducer(bdpt_reducer* r) {
  if (!r) return;
  for (size_t k = 0; k < r->comms.size(); k++)
    if (r->comms[k]) (void)rccl().CommDestroy(r->comms[k]);
  for (size_t k = 0; k < r->scratch.size(); k++)
    if (r->scratch[k]) { (void)hipSetDevice(r->devs[k]); (void)hipFree(r->scratch[k]); }
  // only the reducer's own data from here on: the contexts may already be destroyed
  for (size_t k = 0; k < r->ev.size(); k++)
    if (r->ev[k]) { (void)hipSetDevice(r->ctx_dev[k]); (void)hipEventDestroy(r->ev[k]); }
  for (size_t k = 0; k < r->done.size(); k++)
    if (r->done[k]) { (void)hipSetDevice(r->devs[k]); (void)hipEventDestroy(r->done[k]); }
  delete r;
}

unsigned grid_for(long long n) { return (unsigned)std::max(1LL, std::min<long long>((n / 4 + 255) / 256, 8192)); }

}  // namespace

extern "C" {

int bdpt_reduce_create(void* const* ctxs, int32_t n, bdpt_reducer** out) {
  if (!ctxs || !out || n <= 0) { g_err = "bdpt_reduce_create: null argument or n <= 0"; return BDPT_E_INVALID; }
  *out = nullptr;
  std::unique_ptr<bdpt_reducer, void (*)(bdpt_reducer*)> r(new bdpt_reducer(), free_reducer);
  for (int i = 0; i < n; i++) {
    if (!ctxs[i]) { g_err = "bdpt_reduce_create: null ctx"; return BDPT_E_INVALID; }
    for (int j = 0; j < i; j++)
      if (ctxs[j] == ctxs[i]) { g_err = "bdpt_reduce_create: a ctx is listed twice"; return BDPT_E_INVALID; }
  }
  // every ctx is locked while its fields are read (address order, as bdpt_reduce_frames: a render
  // or clear on another thread waits)
  std::vector<Ctx*> order;
  for (int i = 0; i < n; i++) order.push_back((Ctx*)ctxs[i]);
  std::sort(order.begin(), order.end());
  std::vector<std::unique_lock<std::recursive_mutex>> locks;
  for (Ctx* c : order) locks.emplace_back(c->mu);
  for (int i = 0; i < n; i++) {
    Ctx* c = (Ctx*)ctxs[i];
    if (i > 0 && (c->prm.width != r->ctxs[0]->prm.width || c->prm.height != r->ctxs[0]->prm.height ||
                  c->pt != r->pt)) {
      g_err = "bdpt_reduce_create: every ctx must have the same frame size and integrator";
      return BDPT_E_INVALID;
    }
    if (i == 0) { r->npix = c->npix; r->pt = c->pt; }
    r->ctxs.push_back(c);
    r->ctx_dev.push_back(c->device);
    auto it = std::find(r->devs.begin(), r->devs.end(), c->device);
    if (it == r->devs.end()) {
      r->devs.push_back(c->device);
      r->members.emplace_back();
      it = r->devs.end() - 1;
    }
    const int rank = (int)(it - r->devs.begin());
    r->rank_of.push_back(rank);
    r->members[rank].push_back(i);
  }
  const Rccl& L = rccl();
  if (!L.err.empty()) { g_err = L.err; return BDPT_E_DEVICE; }
  const int nr = (int)r->devs.size();
  r->comms.assign(nr, nullptr);
  r->scratch.assign(nr, nullptr);
  r->ev.assign(n, nullptr);
  NCCLCHK(L.CommInitAll(r->comms.data(), nr, r->devs.data()));
  const size_t n3 = r->npix * 3;
  for (int k = 0; k < nr; k++) {
    HIPCHK(hipSetDevice(r->devs[k]));
    if (r->members[k].size() > 1)
      HIPCHK(hipMalloc((void**)&r->scratch[k], (2 * n3 + r->npix) * sizeof(float)));
  }
  for (int i = 0; i < n; i++) {
    HIPCHK(hipSetDevice(r->ctxs[i]->device));
    HIPCHK(hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming));
  }
  r->done.assign(nr, nullptr);
  for (int k = 0; k < nr; k++) {
    HIPCHK(hipSetDevice(r->devs[k]));
    HIPCHK(hipEventCreateWithFlags(&r->done[k], hipEventDisableTiming));
  }
  *out = r.release();
  return BDPT_OK;
}

int bdpt_reduce_frames(bdpt_reducer* r, int32_t root) {
  if (!r) { g_err = "null reducer"; return BDPT_E_INVALID; }
  const int n = (int)r->ctxs.size();
  if (root < 0 || root >= n) { g_err = "bdpt_reduce_frames: root out of range"; return BDPT_E_INVALID; }
  const Rccl& L = rccl();
  // every ctx is locked for the duration (in address order: no lock-order cycles between callers)
  std::vector<Ctx*> order(r->ctxs);
  std::sort(order.begin(), order.end());
  std::vector<std::unique_lock<std::recursive_mutex>> locks;
  for (Ctx* c : order) locks.emplace_back(c->mu);
  const int nr = (int)r->devs.size();
  const int root_rank = r->rank_of[root];
  Ctx* R = r->ctxs[root];
  const long long n3 = (long long)r->npix * 3, np = (long long)r->npix;
  // per rank: the stream it works on (the root's on the root's device, else its first ctx's) and
  // the buffers it sends
  std::vector<int> lead(nr);
  std::vector<const void*> s_eye(nr), s_light(nr), s_count(nr);
  for (int k = 0; k < nr; k++) {
    lead[k] = k == root_rank ? root : r->members[k][0];
    Ctx* l = r->ctxs[lead[k]];
    HIPCHK(hipSetDevice(r->devs[k]));
    if (r->members[k].size() == 1) {
      s_eye[k] = l->d_eye; s_light[k] = l->d_light; s_count[k] = l->d_count;
      continue;
    }
    // several ctxs on this device: sum them into the scratch pair on the lead's stream, after
    // every member's enqueued work
    float* se = r->scratch[k];
    float* sl = se + n3;
    int* sc = (int*)(sl + n3);
    bool first = true;
    for (int i : r->members[k]) {
      Ctx* c = r->ctxs[i];
      if (i != lead[k]) {
        HIPCHK(hipEventRecord(r->ev[i], c->stream));
        HIPCHK(hipStreamWaitEvent(l->stream, r->ev[i], 0));
      }
      hipLaunchKernelGGL(k_frame_acc, dim3(grid_for(n3)), dim3(256), 0, l->stream, se, c->d_eye, n3, first ? 0 : 1);
      hipLaunchKernelGGL(k_frame_acc, dim3(grid_for(n3)), dim3(256), 0, l->stream, sl, c->d_light, n3, first ? 0 : 1);
      if (r->pt)
        hipLaunchKernelGGL(k_count_acc, dim3(grid_for(np * 4)), dim3(256), 0, l->stream, sc, c->d_count, np, first ? 0 : 1);
      HIPCHK(hipGetLastError());
      first = false;
    }
    s_eye[k] = se; s_light[k] = sl; s_count[k] = sc;
  }
  // the collective: one group, each rank's reduces on its lead stream, into the root's frames.
  // The group is always closed, also when an enqueue fails (an open group would defer every later
  // RCCL call of this thread); the first failure is what the call reports.
  NCCLCHK(L.GroupStart());
  ncclResult_t first = ncclSuccess;
  const char* what = "";
  auto note = [&](ncclResult_t e, const char* call) {
    if (e != ncclSuccess && first == ncclSuccess) { first = e; what = call; }
  };
  for (int k = 0; k < nr && first == ncclSuccess; k++) {
    hipStream_t st = r->ctxs[lead[k]]->stream;
    const bool at_root = k == root_rank;
    note(L.Reduce(s_eye[k], at_root ? R->d_eye : nullptr, (size_t)n3, ncclFloat32, ncclSum, root_rank, r->comms[k], st),
         "ncclReduce (eye frame)");
    note(L.Reduce(s_light[k], at_root ? R->d_light : nullptr, (size_t)n3, ncclFloat32, ncclSum, root_rank, r->comms[k], st),
         "ncclReduce (light frame)");
    if (r->pt)
      note(L.Reduce(s_count[k], at_root ? R->d_count : nullptr, (size_t)np, ncclInt32, ncclSum, root_rank, r->comms[k], st),
           "ncclReduce (sample counts)");
  }
  note(L.GroupEnd(), "ncclGroupEnd");
  if (first != ncclSuccess) {
    g_err = std::string("RCCL ") + what + ": " + L.GetErrorString(first);
    return BDPT_E_DEVICE;
  }
  // later work on any member (a clear, the next render) is ordered after the reduce read its frames
  for (int k = 0; k < nr; k++) {
    Ctx* l = r->ctxs[lead[k]];
    HIPCHK(hipSetDevice(r->devs[k]));
    HIPCHK(hipEventRecord(r->ev[lead[k]], l->stream));
    HIPCHK(hipEventRecord(r->done[k], l->stream));
    for (int i : r->members[k])
      if (i != lead[k]) HIPCHK(hipStreamWaitEvent(r->ctxs[i]->stream, r->ev[lead[k]], 0));
  }
  return BDPT_OK;
}

int bdpt_reduce_ranks(const bdpt_reducer* r) { return r ? (int)r->devs.size() : BDPT_E_INVALID; }

int bdpt_reduce_rccl_version(void) {
  const Rccl& L = rccl();
  if (!L.err.empty()) { g_err = L.err; return BDPT_E_DEVICE; }
  int v = 0;
  NCCLCHK(L.GetVersion(&v));
  return v;
}

void bdpt_reduce_destroy(bdpt_reducer* r) {
  if (!r) return;
  // finish the last reduce (its device sums and collectives, which use the scratch freed below)
  // through the reducer's own events: the contexts may already be destroyed (bdpt_destroy syncs
  // its stream first, so their part of the work has completed then)
  for (size_t k = 0; k < r->devs.size(); k++) {
    (void)hipSetDevice(r->devs[k]);
    if (r->done[k]) (void)hipEventSynchronize(r->done[k]);
  }
  free_reducer(r);
}

}  // extern "C"
