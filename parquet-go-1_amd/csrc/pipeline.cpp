// pipeline.cpp — streaming row-group decode (pqgpu_pipeline_*, include/pqgpu.h).
//
// The reference reads a file row group by row group (FileReader.readRowGroupData,
// chunk_reader.go:375-404, from the NextRow / PreLoad loop, file_reader.go:187-198) and decodes
// each chunk's pages on the calling goroutine. Here every row group is one batch; `depth`
// batches rotate through slots, each with its own HIP stream and events:
//
//   worker thread (host):  reset -> add_file_chunk x columns (page-header walk, GZIP/dictionary
//                          pages, staging) -> upload (descriptors + pinned copy, H2D enqueued)
//                          -> decode (kernels enqueued)            [slot stream]
//   caller (next):         wait for its row group's slot -> sync (errors, counts) -> hand out
//   caller (release):      slot free again -> a worker plans row group k + depth into it
//
// so the host work and the H2D copy of later row groups overlap the GPU decode of earlier
// ones. Row groups are claimed in order; the caller receives them in order.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pqgpu.h"
#include "ctx.h"

namespace {

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

enum SlotState { FREE, PLANNING, LAUNCHED, OUT };

struct Slot {
  pqgpu_batch *b = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;  // upload start, upload done, decode done
  SlotState state = FREE;
  int64_t index = -1;  // row-group position in the pipeline's list
  int rc = PQ_OK;      // first launch error (upload / decode)
  pqgpu_error err{};
  // device_index: the row group's byte range, staged in pinned memory and resident on the device
  void *h_raw = nullptr, *d_raw = nullptr;
  size_t raw_cap = 0;
};

void set_err(pqgpu_error *e, int code, const char *msg) {
  if (!e) return;
  e->code = code;
  e->chunk = -1;
  e->page = -1;
  snprintf(e->msg, sizeof(e->msg), "%s", msg);
}

}  // namespace

struct pqgpu_pipeline {
  pqgpu_ctx *ctx = nullptr;
  const pqgpu_file *f = nullptr;
  std::vector<int32_t> rgs, cols;
  int validate_crc = 0, device_index = 0;
  bool registered = false;  // device_index: the file buffer is page-locked (H2D straight from it)
  std::vector<Slot> slots;
  std::vector<std::thread> workers;
  std::mutex m;
  std::condition_variable cv;
  int64_t next_plan = 0, next_out = 0;
  bool stop = false;
  clk::time_point t0;
  pqgpu_pipeline_stats st{};
};

// device_index: copy the selected chunks' byte range of row group `rg` to the slot's device buffer
// (through its pinned staging buffer) and walk their page headers there. nullptr: walk on the host.
static pqgpu_page_index *index_row_group(pqgpu_pipeline *p, Slot *sl, int32_t rg) {
  std::vector<pqgpu_chunk_meta> metas(p->cols.size());
  int64_t lo = INT64_MAX, hi = 0;
  const int64_t flen = (int64_t)pqgpu_file_len(p->f);
  for (size_t k = 0; k < p->cols.size(); k++) {
    pqgpu_error e;
    if (pqgpu_file_chunk_meta(p->f, rg, p->cols[k], &metas[k], &e)) return nullptr;  // the host path reports it
    const pqgpu_chunk_meta &m = metas[k];
    const int64_t st = m.dictionary_page_offset >= 0 ? m.dictionary_page_offset : m.data_page_offset;
    lo = std::min(lo, std::max<int64_t>(st, 0));
    hi = std::max(hi, std::min(flen, st + std::max<int64_t>(m.total_compressed_size, 0)));
  }
  if (lo >= hi) return nullptr;
  const size_t n = (size_t)(hi - lo);
  if (n + 64 > sl->raw_cap) {
    if (sl->h_raw) (void)hipHostFree(sl->h_raw);
    if (sl->d_raw) (void)hipFree(sl->d_raw);
    sl->h_raw = sl->d_raw = nullptr;
    sl->raw_cap = 0;
    const size_t cap = n + n / 8 + 4096;
    if ((!p->registered && hipHostMalloc(&sl->h_raw, cap, hipHostMallocDefault) != hipSuccess) ||
        hipMalloc(&sl->d_raw, cap) != hipSuccess)
      return nullptr;
    sl->raw_cap = cap;
  }
  const uint8_t *src = pqgpu_file_bytes(p->f) + lo;
  if (!p->registered) {  // stage through the slot's pinned buffer
    memcpy(sl->h_raw, src, n);
    src = (const uint8_t *)sl->h_raw;
  }
  if (hipMemcpyAsync(sl->d_raw, src, n, hipMemcpyHostToDevice, sl->s) != hipSuccess) return nullptr;
  pqgpu_page_index *ix = nullptr;
  pqgpu_error e;
  if (pqgpu_page_index_build(p->ctx, sl->d_raw, lo, (int64_t)n, metas.data(), (int32_t)metas.size(), p->validate_crc,
                             sl->s, &ix, &e))
    return nullptr;
  return ix;
}

static void worker(pqgpu_pipeline *p) {
  (void)hipSetDevice(p->ctx->device);
  const int64_t n = (int64_t)p->rgs.size(), depth = (int64_t)p->slots.size();
  for (;;) {
    int64_t i;
    Slot *sl;
    {
      std::unique_lock<std::mutex> lk(p->m);
      // claim the next row group once its slot is free (the slot's previous row group released)
      p->cv.wait(lk, [&] {
        return p->stop || p->next_plan >= n || p->slots[(size_t)(p->next_plan % depth)].state == FREE;
      });
      if (p->stop || p->next_plan >= n) return;
      i = p->next_plan++;
      sl = &p->slots[(size_t)(i % depth)];
      sl->state = PLANNING;
      sl->index = i;
    }
    const auto tp = clk::now();
    pqgpu_batch_reset(sl->b);
    sl->rc = PQ_OK;
    memset(&sl->err, 0, sizeof(sl->err));
    const int32_t rg = p->rgs[(size_t)i];
    pqgpu_page_index *ix = p->device_index ? index_row_group(p, sl, rg) : nullptr;
    const double ixms = ix ? ms_since(tp) : 0.0;
    int32_t ix_polls = 0, ix_unrep = 0, ix_fb = 0, ix_stale = 0;
    if (ix) (void)pqgpu_page_index_stats(ix, &ix_polls, &ix_unrep, &ix_fb, nullptr, &ix_stale);
    for (size_t k = 0; k < p->cols.size(); k++) {
      int32_t id;
      pqgpu_error e;
      if (ix)  // page headers (and checksums) walked on the device; chunks it did not take fall back
        (void)pqgpu_batch_add_indexed_file_chunk(sl->b, ix, (int32_t)k, p->f, p->cols[k], p->validate_crc, &id, &e);
      else
        (void)pqgpu_batch_add_file_chunk(sl->b, p->f, rg, p->cols[k], p->validate_crc, &id, &e);  // errors stay per chunk
    }
    const double plan = ms_since(tp);
    const auto tu = clk::now();
    (void)hipEventRecord(sl->e0, sl->s);
    int rc = pqgpu_batch_upload(sl->b, sl->s, &sl->err);  // gathers resident pages; returns when done
    const double up = ms_since(tu);
    pqgpu_page_index_destroy(ix);
    (void)hipEventRecord(sl->e1, sl->s);
    if (!rc) rc = pqgpu_batch_decode(sl->b, sl->s, &sl->err);
    (void)hipEventRecord(sl->e2, sl->s);
    {
      std::lock_guard<std::mutex> lk(p->m);
      sl->rc = rc;
      sl->state = LAUNCHED;
      p->st.plan_ms += plan;
      p->st.index_ms += ixms;
      p->st.ix_polls += ix_polls;
      p->st.ix_unreported += ix_unrep;
      p->st.ix_fallback_chunks += ix_fb;
      p->st.ix_stale_entries += ix_stale;
      p->st.upload_ms += up;
    }
    p->cv.notify_all();
  }
}

static void destroy(pqgpu_pipeline *p) {
  {
    std::lock_guard<std::mutex> lk(p->m);
    p->stop = true;
  }
  p->cv.notify_all();
  for (auto &t : p->workers) t.join();
  (void)hipSetDevice(p->ctx->device);
  for (auto &sl : p->slots) {
    if (sl.s) (void)hipStreamSynchronize(sl.s);
    if (sl.b) pqgpu_batch_destroy(sl.b);
    if (sl.e0) (void)hipEventDestroy(sl.e0);
    if (sl.e1) (void)hipEventDestroy(sl.e1);
    if (sl.e2) (void)hipEventDestroy(sl.e2);
    if (sl.h_raw) (void)hipHostFree(sl.h_raw);
    if (sl.d_raw) (void)hipFree(sl.d_raw);
    if (sl.s) (void)hipStreamDestroy(sl.s);
  }
  if (p->registered) (void)hipHostUnregister((void *)pqgpu_file_bytes(p->f));
  delete p;
}

extern "C" int pqgpu_pipeline_create(pqgpu_ctx *ctx, const pqgpu_file *f, const int32_t *rgs, int32_t n_rgs,
                                     const int32_t *cols, int32_t n_cols, const pqgpu_pipeline_opts *opts,
                                     pqgpu_pipeline **out, pqgpu_error *err) {
  if (out) *out = nullptr;
  if (!ctx || !f || !out) {
    set_err(err, PQ_ERR_ARG, "pipeline needs a device context, a file and an output pointer");
    return PQ_ERR_ARG;
  }
  const int nrg = pqgpu_file_num_row_groups(f), ncol = pqgpu_file_num_columns(f);
  pqgpu_pipeline *p = new pqgpu_pipeline();
  p->ctx = ctx;
  p->f = f;
  for (int32_t k = 0; k < (rgs ? n_rgs : nrg); k++) p->rgs.push_back(rgs ? rgs[k] : k);
  for (int32_t k = 0; k < (cols ? n_cols : ncol); k++) p->cols.push_back(cols ? cols[k] : k);
  for (int32_t r : p->rgs)
    if (r < 0 || r >= nrg) { delete p; set_err(err, PQ_ERR_ARG, "row group out of range"); return PQ_ERR_ARG; }
  for (int32_t c : p->cols)
    if (c < 0 || c >= ncol) { delete p; set_err(err, PQ_ERR_ARG, "column out of range"); return PQ_ERR_ARG; }
  const int depth = opts && opts->depth > 0 ? opts->depth : 3;
  const int threads = opts && opts->threads > 0 ? opts->threads : depth;
  p->validate_crc = opts ? opts->validate_crc : 0;
  p->device_index = opts ? opts->device_index : 0;
  // device_index copies whole row-group ranges H2D: page-lock the file buffer once so they go
  // straight from it (a buffer that cannot be registered, e.g. already pinned, is staged instead)
  if (p->device_index && pqgpu_file_len(f) > 0 && hipSetDevice(ctx->device) == hipSuccess)
    p->registered = hipHostRegister((void *)pqgpu_file_bytes(f), pqgpu_file_len(f), hipHostRegisterDefault) == hipSuccess;
  if (p->device_index && !p->registered) (void)hipGetLastError();
  if (hipSetDevice(ctx->device) != hipSuccess) { delete p; set_err(err, PQ_ERR_HIP, "hipSetDevice failed"); return PQ_ERR_HIP; }
  p->slots.resize((size_t)depth);
  for (auto &sl : p->slots) {
    pqgpu_error e;
    if (pqgpu_batch_create(ctx, &sl.b, &e) || hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&sl.e0) != hipSuccess || hipEventCreate(&sl.e1) != hipSuccess ||
        hipEventCreate(&sl.e2) != hipSuccess) {
      destroy(p);
      set_err(err, PQ_ERR_HIP, "pipeline: batch / stream / event creation failed");
      return PQ_ERR_HIP;
    }
  }
  p->t0 = clk::now();
  for (int k = 0; k < threads; k++) p->workers.emplace_back(worker, p);
  *out = p;
  return PQ_OK;
}

extern "C" int pqgpu_pipeline_next(pqgpu_pipeline *p, pqgpu_batch **batch, int32_t *rg, pqgpu_error *err) {
  if (err) memset(err, 0, sizeof(*err)), err->chunk = err->page = -1;
  *batch = nullptr;
  if (rg) *rg = -1;
  const int64_t n = (int64_t)p->rgs.size(), depth = (int64_t)p->slots.size();
  Slot *sl;
  int64_t i;
  {
    std::unique_lock<std::mutex> lk(p->m);
    i = p->next_out;
    if (i >= n) return PQ_OK;
    sl = &p->slots[(size_t)(i % depth)];
    if (sl->state == OUT) {  // its slot still holds row group i - depth: it would never be planned
      set_err(err, PQ_ERR_ARG, "pipeline: release the previous row groups' batches before asking for more");
      return PQ_ERR_ARG;
    }
    p->cv.wait(lk, [&] { return sl->state == LAUNCHED && sl->index == i; });
  }
  int rc = sl->rc;
  if (rc) {
    if (err) *err = sl->err;
    (void)hipStreamSynchronize(sl->s);
  } else {
    rc = pqgpu_batch_sync(sl->b, sl->s, err);
  }
  float h2d = 0, dec = 0;
  (void)hipEventElapsedTime(&h2d, sl->e0, sl->e1);
  (void)hipEventElapsedTime(&dec, sl->e1, sl->e2);
  pqgpu_batch_stats bs;
  pqgpu_batch_stats_get(sl->b, &bs);
  {
    std::lock_guard<std::mutex> lk(p->m);
    sl->state = OUT;
    p->next_out++;
    p->st.row_groups++;
    p->st.rows += pqgpu_file_row_group_num_rows(p->f, p->rgs[(size_t)i]);
    p->st.chunks += (int64_t)p->cols.size();
    for (int c = 0; c < pqgpu_batch_num_chunks(sl->b); c++)
      if (pqgpu_batch_chunk_status(sl->b, c, nullptr)) p->st.failed_chunks++;
    p->st.input_bytes += bs.staged_bytes;
    p->st.output_bytes += bs.output_bytes;
    p->st.h2d_ms += h2d;
    p->st.decode_ms += dec;
    p->st.wall_ms = ms_since(p->t0);
  }
  *batch = sl->b;
  if (rg) *rg = p->rgs[(size_t)i];
  return rc;
}

extern "C" int pqgpu_pipeline_release(pqgpu_pipeline *p, pqgpu_batch *batch) {
  {
    std::lock_guard<std::mutex> lk(p->m);
    bool found = false;
    for (auto &sl : p->slots)
      if (sl.b == batch && sl.state == OUT) { sl.state = FREE; found = true; }
    if (!found) return PQ_ERR_ARG;
  }
  p->cv.notify_all();
  return PQ_OK;
}

extern "C" int pqgpu_pipeline_stats_get(const pqgpu_pipeline *p, pqgpu_pipeline_stats *out) {
  std::lock_guard<std::mutex> lk(const_cast<pqgpu_pipeline *>(p)->m);
  *out = p->st;
  return PQ_OK;
}

extern "C" void pqgpu_pipeline_destroy(pqgpu_pipeline *p) {
  if (p) destroy(p);
}
