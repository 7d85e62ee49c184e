// Host -> device span upload (the product path's one conversion per
// experiment: collect_trace.sh:70 converts each dump once, then every feature
// is computed from it): DMA from the caller's registered pages, with a pinned
// staging pipeline as the fallback (history below).
//
// r04 uploaded with pageable hipMemcpyAsync calls after two serial host passes
// (the max-service scan and a fresh svc|flags packing vector): 108.9 ms for
// 55.6 M spans, 98 % of it host work.  Here the columns
// are cut into 8-MiB pieces dealt round-robin to W worker threads; each
// worker copies (or packs svc|flags, taking the largest service on the way)
// its piece into one of its two pinned buffers and hands it to the DMA on its
// own stream, so host copies, packing and PCIe transfers overlap and the
// DMA sees W streams at once.  The workers, their streams and pinned
// buffers live with the ctx.
//
// r06: a plain column (kind 0) no longer goes through a bounce buffer: it is
// registered with the driver for the call (hipHostRegister, ~2 ms per GB the
// first time, then ~0.02 ms; unregistered before the call returns, so no
// registration outlives the caller's buffer) and copied by the DMA engine
// straight from the caller's pages on the ctx stream — 53 GB/s on the GPU box
// against 33 GB/s through the bounce (scripts/r06/time_upload.py: more
// concurrent DMA streams from registered memory measured slower, 21-28 GB/s
// at 8).  svc|flags (kind 1) goes the same way: its two u16 columns are
// copied into a device scratch and packed there by pack_svc_flags_kernel,
// which also takes the largest service.  Items under a piece are copied from
// pageable memory (svc|flags packed on the host first).  So the pipeline of
// worker threads and pinned buffers (~0.1 s to create: the first host call's
// cost in r05 / early r06) is made only for a column the driver refuses to
// register, or when ANOMOD_UPLOAD_DIRECT=0 asks for it.
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "common.h"

namespace anomod {

#ifdef ANOMOD_UPLOAD_TIMING  // step times to stderr (timing-only builds, scripts/r06)
void ut_mark(const char* step) {
  static double last = host_now_ms();
  const double now = host_now_ms();
  fprintf(stderr, "upload %-28s %8.2f ms\n", step, now - last);
  last = now;
}
#define UT_MARK(step) ut_mark(step)
#else
#define UT_MARK(step) ((void)0)
#endif

struct Uploader {
  static constexpr size_t kPiece = size_t(8) << 20;  // bytes of device data per piece
  struct Piece {
    int item;
    uint64_t off, len;  // in the item's units (bytes, or packed elements)
  };
  int device = 0, nw = 0;
  std::vector<std::thread> th;
  std::vector<hipStream_t> st;
  hipStream_t shared = nullptr;  // the workers' one DMA stream beside direct copies
  bool one_stream = false;       // this call: workers' DMAs on `shared`
  std::vector<void*> pin;       // two per worker
  std::vector<hipEvent_t> ev;   // two per worker
  std::mutex m;
  std::condition_variable cv_go, cv_done;
  uint64_t gen = 0;
  int pending = 0;
  bool quit = false;
  const UpItem* items = nullptr;
  std::vector<Piece> pieces;
  std::vector<uint32_t> wmax;
  std::vector<hipError_t> werr;

  // Beside direct copies the workers' DMAs share one stream: registered
  // memory measured 53 GB/s on 1-4 concurrent DMA streams and 21-28 GB/s on 8.
  hipStream_t stream(int w) const { return one_stream ? shared : st[w]; }

  void work(int w) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m);
        cv_go.wait(lk, [&] { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
      }
      hipError_t err = hipSetDevice(device);
      uint32_t mx = 0;
      int slot = 0;
      for (size_t i = (size_t)w; err == hipSuccess && i < pieces.size(); i += (size_t)nw) {
        const Piece& P = pieces[i];
        const UpItem& it = items[P.item];
        void* buf = pin[2 * w + slot];
        err = hipEventSynchronize(ev[2 * w + slot]);  // the DMA out of this buffer is done
        if (err != hipSuccess) break;
        size_t bytes;
        char* dst;
        if (it.kind == 1) {  // svc (u16) | flags (u16) << 16 -> u32
          const uint16_t* svc = static_cast<const uint16_t*>(it.a) + P.off;
          const uint16_t* fl = static_cast<const uint16_t*>(it.b) + P.off;
          uint32_t* o = static_cast<uint32_t*>(buf);
          for (uint64_t j = 0; j < P.len; ++j) {
            o[j] = (uint32_t)svc[j] | ((uint32_t)fl[j] << 16);
            mx = svc[j] > mx ? svc[j] : mx;
          }
          bytes = P.len * 4;
          dst = static_cast<char*>(it.dst) + P.off * 4;
        } else {
          std::memcpy(buf, static_cast<const char*>(it.a) + P.off, P.len);
          bytes = P.len;
          dst = static_cast<char*>(it.dst) + P.off;
        }
        err = hipMemcpyAsync(dst, buf, bytes, hipMemcpyHostToDevice, stream(w));
        if (err == hipSuccess) err = hipEventRecord(ev[2 * w + slot], stream(w));
        slot ^= 1;
      }
      const hipError_t e2 = hipStreamSynchronize(stream(w));
      if (err == hipSuccess) err = e2;
      std::lock_guard<std::mutex> lk(m);
      wmax[w] = mx;
      werr[w] = err;
      if (--pending == 0) cv_done.notify_one();
    }
  }
};

namespace {

int make_uploader(anomod_ctx* ctx) {
  if (ctx->uploader) return ANOMOD_OK;
  const double t0 = host_now_ms();
  auto* u = new Uploader();
  u->device = ctx->device;
  const char* e = std::getenv("ANOMOD_UPLOAD_THREADS");
  int nw = e && *e ? std::atoi(e) : 8;
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw) nw = std::min<int>(nw, (int)hw);
  nw = std::max(1, std::min(nw, 32));
  u->nw = nw;
  u->st.assign(nw, nullptr);
  u->pin.assign(2 * nw, nullptr);
  u->ev.assign(2 * nw, nullptr);
  u->wmax.assign(nw, 0u);
  u->werr.assign(nw, hipSuccess);
  bool ok = true;
  ok = hipStreamCreateWithFlags(&u->shared, hipStreamNonBlocking) == hipSuccess;
  for (int w = 0; ok && w < nw; ++w) {
    ok = hipStreamCreateWithFlags(&u->st[w], hipStreamNonBlocking) == hipSuccess;
    for (int s = 0; ok && s < 2; ++s) {
      ok = hipHostMalloc(&u->pin[2 * w + s], Uploader::kPiece, hipHostMallocDefault) == hipSuccess &&
           hipEventCreateWithFlags(&u->ev[2 * w + s], hipEventDisableTiming) == hipSuccess;
    }
  }
  ctx->uploader = u;  // (freed by free_uploader on failure too)
  if (!ok) {
    free_uploader(ctx);
    set_error(ctx, "creating the upload pipeline (%d pinned 2 x 8-MiB buffers) failed", nw);
    return ANOMOD_ENOMEM;
  }
  for (int w = 0; w < nw; ++w) u->th.emplace_back([u, w] { u->work(w); });
  host_record(ctx, kHostUploadSetup, host_now_ms() - t0);
  return ANOMOD_OK;
}

}  // namespace

void free_uploader(anomod_ctx* ctx) {
  Uploader* u = ctx->uploader;
  if (!u) return;
  {
    std::lock_guard<std::mutex> lk(u->m);
    u->quit = true;
  }
  u->cv_go.notify_all();
  for (auto& t : u->th) t.join();
  for (auto s : u->st)
    if (s) (void)hipStreamDestroy(s);
  if (u->shared) (void)hipStreamDestroy(u->shared);
  for (auto p : u->pin)
    if (p) (void)hipHostFree(p);
  for (auto e : u->ev)
    if (e) (void)hipEventDestroy(e);
  delete u;
  ctx->uploader = nullptr;
}

namespace {

// svc (u16) | flags (u16) << 16 -> u32, and the largest service (atomic max
// of the waves' maxima into *mx)
__global__ __launch_bounds__(256) void pack_svc_flags_kernel(const uint16_t* __restrict__ svc,
                                                             const uint16_t* __restrict__ fl,
                                                             uint32_t* __restrict__ out, uint64_t n,
                                                             unsigned int* __restrict__ mx) {
  uint32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * 256u) {
    const uint32_t s = svc[i];
    out[i] = s | ((uint32_t)fl[i] << 16);
    m = s > m ? s : m;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)m, o);
    m = y > m ? y : m;
  }
  if ((threadIdx.x & 63u) == 0 && m) atomicMax(mx, m);
}

}  // namespace

int upload_items(anomod_ctx* ctx, const UpItem* items, int n_items, uint32_t* max_svc) {
  if (max_svc) *max_svc = 0;
  uint64_t total = 0;
  for (int i = 0; i < n_items; ++i) total += items[i].n;
  if (total == 0) return ANOMOD_OK;
  // the ctx stream's earlier work on these buffers (a previous call's kernels
  // reading a reused set) must be done before other streams write them
  ANOMOD_HIP(ctx, hipStreamSynchronize(ctx->stream));
  UT_MARK("enter + stream sync");
  const char* de = getenv("ANOMOD_UPLOAD_DIRECT");
  const bool direct_ok = !(de && de[0] == '0');
  std::vector<const void*> registered;
  std::vector<char> done(n_items, 0);
  std::vector<std::vector<uint32_t>> packed;  // small svc|flags items, packed on the host
  uint32_t mx = 0;
  unsigned int* d_mx = nullptr;  // the device pack's largest service
  hipError_t err = hipSuccess;
  // any refusal (read-only pages, a page another column registered first,
  // memory the caller pinned) leaves the item to the bounce pipeline: a range
  // only partly registered must never be handed to the DMA engine
  auto reg = [&](const void* a, uint64_t bytes) {
    if (hipHostRegister(const_cast<void*>(a), bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    registered.push_back(a);
    return true;
  };
  auto unreg_last = [&]() {
    (void)hipHostUnregister(const_cast<void*>(registered.back()));
    registered.pop_back();
  };
  for (int i = 0; direct_ok && err == hipSuccess && i < n_items; ++i) {
    const UpItem& it = items[i];
    const uint64_t bytes = it.kind == 1 ? it.n * 4 : it.n;
    if (bytes == 0) {
      done[i] = 1;
      continue;
    }
    if (bytes < Uploader::kPiece) {  // small: from pageable memory
      if (it.kind == 0) {
        err = hipMemcpyAsync(it.dst, it.a, it.n, hipMemcpyHostToDevice, ctx->stream);
      } else {
        packed.emplace_back(it.n);
        const auto* sv = static_cast<const uint16_t*>(it.a);
        const auto* fl = static_cast<const uint16_t*>(it.b);
        uint32_t* o = packed.back().data();
        for (uint64_t j = 0; j < it.n; ++j) {
          o[j] = (uint32_t)sv[j] | ((uint32_t)fl[j] << 16);
          mx = sv[j] > mx ? sv[j] : mx;
        }
        err = hipMemcpyAsync(it.dst, o, bytes, hipMemcpyHostToDevice, ctx->stream);
      }
      done[i] = 1;
      continue;
    }
    if (it.kind == 0) {
      if (!reg(it.a, it.n)) continue;
      UT_MARK("register column");
      err = hipMemcpyAsync(it.dst, it.a, it.n, hipMemcpyHostToDevice, ctx->stream);
      UT_MARK("issue copy");
      done[i] = 1;
      continue;
    }
    // svc | flags: both u16 columns registered and copied into the scratch,
    // packed on the device (one such item per call: the scratch holds one)
    if (d_mx) continue;
    if (!reg(it.a, it.n * 2)) continue;
    if (!reg(it.b, it.n * 2)) {
      unreg_last();
      continue;
    }
    UT_MARK("register svc + flags");
    void* scr = nullptr;
    const uint64_t half = (it.n * 2 + 255) & ~255ull;
    if (ensure_scratch(ctx, kScratchUpload, 2 * half + 256, &scr) != ANOMOD_OK) {
      unreg_last();
      unreg_last();
      continue;
    }
    UT_MARK("scratch");
    char* base = static_cast<char*>(scr);
    auto* dsv = reinterpret_cast<uint16_t*>(base);
    auto* dfl = reinterpret_cast<uint16_t*>(base + half);
    d_mx = reinterpret_cast<unsigned int*>(base + 2 * half);
    err = hipMemcpyAsync(dsv, it.a, it.n * 2, hipMemcpyHostToDevice, ctx->stream);
    if (err == hipSuccess)
      err = hipMemcpyAsync(dfl, it.b, it.n * 2, hipMemcpyHostToDevice, ctx->stream);
    if (err == hipSuccess) err = hipMemsetAsync(d_mx, 0, 4, ctx->stream);
    if (err == hipSuccess) {
      const uint64_t blocks = std::min<uint64_t>((it.n + 255) / 256, (uint64_t)ctx->num_cus * 8);
      hipLaunchKernelGGL(pack_svc_flags_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream,
                         dsv, dfl, static_cast<uint32_t*>(it.dst), it.n, d_mx);
      err = hipGetLastError();
    }
    UT_MARK("issue svc/flags + pack");
    done[i] = 1;
  }
  // the rest (a refused registration, or ANOMOD_UPLOAD_DIRECT=0): the bounce
  // pipeline, its DMAs on one stream beside the ctx stream's direct copies
  bool rest = false;
  for (int i = 0; i < n_items; ++i) rest = rest || !done[i];
  Uploader* u = nullptr;
  if (rest && err == hipSuccess) {
    if (int rc = make_uploader(ctx)) {
      (void)hipStreamSynchronize(ctx->stream);
      for (const void* a : registered) (void)hipHostUnregister(const_cast<void*>(a));
      return rc;
    }
    u = ctx->uploader;
    u->pieces.clear();
    for (int i = 0; i < n_items; ++i) {
      if (done[i]) continue;
      const uint64_t unit = items[i].kind == 1 ? Uploader::kPiece / 4 : Uploader::kPiece;
      for (uint64_t off = 0; off < items[i].n; off += unit)
        u->pieces.push_back({i, off, std::min<uint64_t>(unit, items[i].n - off)});
    }
    std::unique_lock<std::mutex> lk(u->m);
    u->one_stream = done != std::vector<char>(n_items, 0);
    u->items = items;
    u->pending = u->nw;
    ++u->gen;
    u->cv_go.notify_all();
    u->cv_done.wait(lk, [&] { return u->pending == 0; });
  }
  const hipError_t sync = hipStreamSynchronize(ctx->stream);
  if (err == hipSuccess) err = sync;
  UT_MARK("sync (copies done)");
  uint32_t dmx = 0;
  if (err == hipSuccess && d_mx) err = hipMemcpy(&dmx, d_mx, 4, hipMemcpyDeviceToHost);
  for (const void* a : registered) (void)hipHostUnregister(const_cast<void*>(a));
  UT_MARK("max readback + unregister");
  if (err != hipSuccess) {
    set_error(ctx, "span upload failed: %s", hipGetErrorString(err));
    return ANOMOD_EHIP;
  }
  mx = std::max(mx, dmx);
  for (int w = 0; u && w < u->nw; ++w) {
    if (u->werr[w] != hipSuccess) {
      set_error(ctx, "span upload failed: %s", hipGetErrorString(u->werr[w]));
      return ANOMOD_EHIP;
    }
    mx = std::max(mx, u->wmax[w]);
  }
  if (max_svc) *max_svc = mx;
  return ANOMOD_OK;
}

}  // namespace anomod
