// drawpipe.hip — the replay learning loop's NumPy-exact draws made ahead on a native thread
// (learning._replay_pipelined; host code only, no kernels).
//
// The reference draws, per reshuffle, SWR_divide's rows (make_exps.py:123-125 ->
// compute_stats.py:48-54: N randint calls on [0, n_X) of kx values, then N on [0, n_Z)), and per
// step grad_inc_block's pairs (compute_stats.py:155-156) — one MT19937 stream, NumPy's global
// RandomState, advanced in place here (key/pos point into it).  The loop's segments (runs of
// steps between evaluations) are drawn in order into a ring of pinned host buffers — a
// segment's pairs, and the row tables of every reshuffle inside it, in the reference's draw
// order (a reshuffle's rows before the pairs of its step);
// the main thread waits for segment j, ships it (one upload kernel reading the pinned buffer)
// and records that upload on its stream; the worker refills a buffer only after the upload out
// of it has run (hipEventSynchronize on the recorded event).  A Python worker thread did the
// same with ~60 us per 25-step segment of interpreter and GIL overhead on top of the draws.
#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "tw_common.h"

namespace tw {
namespace {

struct DrawPipe {
  uint32_t* key;
  int32_t* pos;
  std::vector<int32_t> steps;
  std::vector<int32_t> phase;  // step of the reshuffle period at each segment's first step
  int64_t mod;                 // reshuffle period (steps)
  int32_t row_tabs;            // row tables per row buffer
  int32_t row_width;           // bytes per row value: 8 (int64) or 2 (uint16)
  int32_t N;
  int64_t kx, kz, B, n_X, n_Z;
  int32_t width, nbuf;
  std::vector<void*> seg_bufs;
  std::vector<char*> row_bufs;
  std::vector<hipEvent_t> shipped_ev;
  std::vector<int64_t> row_low, row_high, row_cnt;

  std::mutex mu;
  std::condition_variable cv;
  int32_t drawn = 0;    // segments [0, drawn) are in their buffers
  int32_t shipped = 0;  // segments [0, shipped) have their upload recorded
  int rc = TW_OK;       // the first failing draw's status (the worker stops there)
  bool cancel = false;
  std::thread worker;

  void run() {
    const int32_t n_seg = (int32_t)steps.size();
    for (int32_t j = 0; j < n_seg; ++j) {
      const int k = j % nbuf;
      if (j >= nbuf) {  // buffer k held segment j - nbuf: wait until its upload has run
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return cancel || shipped > j - nbuf; });
        if (cancel) return;
        lk.unlock();
        if (hipEventSynchronize(shipped_ev[k]) != hipSuccess) {
          finish(TW_ERR_HIP);
          return;
        }
      }
      int r = 0, tabs = 0;
      const int64_t per = 2 * (int64_t)N * B, wtab = (int64_t)N * (kx + kz);
      for (int32_t k0 = 0; k0 < steps[j] && !r;) {
        const int64_t ph = ((int64_t)phase[j] + k0) % mod;
        if (ph == 0) {  // a reshuffle at this step: its rows first (SWR_divide, then the pairs)
          if (tabs == row_tabs) {
            r = 1;
            break;
          }
          char* dst = row_bufs[k] + (int64_t)tabs * wtab * row_width;
          r = row_width == 2
                  ? tw_np_randint_batch_u16(key, pos, 2 * N, row_low.data(), row_high.data(),
                                            row_cnt.data(), (uint16_t*)dst)
                  : tw_np_randint_batch(key, pos, 2 * N, row_low.data(), row_high.data(),
                                        row_cnt.data(), (int64_t*)dst);
          ++tabs;
          if (r) break;
        }
        const int32_t run = (int32_t)std::min<int64_t>(steps[j] - k0, mod - ph);
        const int64_t at = (int64_t)k0 * per;
        if (width == 1)
          r = tw_np_randint_pairs_steps_u8(key, pos, run, N, kx, kz, B,
                                           (uint8_t*)seg_bufs[k] + at);
        else if (width == 2)
          r = tw_np_randint_pairs_steps_u16(key, pos, run, N, kx, kz, B,
                                            (uint16_t*)seg_bufs[k] + at);
        else
          r = tw_np_randint_pairs_steps(key, pos, run, N, kx, kz, B, (int64_t*)seg_bufs[k] + at);
        k0 += run;
      }
      if (r) {
        finish(TW_ERR_ARG);
        return;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        drawn = j + 1;
      }
      cv.notify_all();
    }
  }

  void finish(int status) {
    {
      std::lock_guard<std::mutex> lk(mu);
      rc = status;
      cancel = true;
    }
    cv.notify_all();
  }
};

}  // namespace
}  // namespace tw

extern "C" int tw_draw_pipe_start(uint32_t* key, int32_t* pos, int32_t n_seg,
                                  const int32_t* seg_steps, const int32_t* seg_phase,
                                  int64_t mod, int32_t N, int64_t kx, int64_t kz, int64_t B,
                                  int64_t n_X, int64_t n_Z, int32_t width, int32_t nbuf,
                                  void* const* seg_bufs, void* const* row_bufs,
                                  int32_t row_tabs, int32_t row_width, void** out_handle) {
  TW_ARG_CHECK(key && pos && out_handle && n_seg >= 0 && N >= 0 && B >= 0 && mod >= 1 &&
                   row_tabs >= 1 && (n_seg == 0 || (seg_steps && seg_phase)),
               "tw_draw_pipe_start: bad arguments");
  for (int32_t j = 0; j < n_seg; ++j)
    TW_ARG_CHECK(seg_steps[j] >= 0 && seg_phase[j] >= 0 && seg_phase[j] < mod,
                 "tw_draw_pipe_start: segment %d: steps %d, phase %d (mod %lld)", j,
                 seg_steps[j], seg_phase[j], (long long)mod);
  TW_ARG_CHECK(nbuf >= 1 && nbuf <= 16 && seg_bufs && row_bufs, "tw_draw_pipe_start: buffers");
  TW_ARG_CHECK(width == 1 || width == 2 || width == 8, "tw_draw_pipe_start: width 1, 2 or 8");
  TW_ARG_CHECK(kx >= 1 && kz >= 1 && n_X >= 1 && n_Z >= 1, "tw_draw_pipe_start: empty ranges");
  TW_ARG_CHECK(row_width == 8 || (row_width == 2 && n_X <= 65536 && n_Z <= 65536),
               "tw_draw_pipe_start: row width %d (uint16 rows need n_X, n_Z <= 65536)",
               row_width);
  TW_ARG_CHECK((width != 1 || (kx <= 256 && kz <= 256)) &&
                   (width != 2 || (kx <= 65536 && kz <= 65536)),
               "tw_draw_pipe_start: indices do not fit the width");
  auto* p = new tw::DrawPipe();
  p->key = key;
  p->pos = pos;
  p->steps.assign(seg_steps, seg_steps + n_seg);
  p->phase.assign(seg_phase, seg_phase + n_seg);
  p->mod = mod;
  p->row_tabs = row_tabs;
  p->row_width = row_width;
  p->N = N;
  p->kx = kx;
  p->kz = kz;
  p->B = B;
  p->n_X = n_X;
  p->n_Z = n_Z;
  p->width = width;
  p->nbuf = nbuf;
  p->seg_bufs.assign(seg_bufs, seg_bufs + nbuf);
  for (int k = 0; k < nbuf; ++k) p->row_bufs.push_back((char*)row_bufs[k]);
  // SWR_divide's calls: N on [0, n_X) of n_X / N values, then N on [0, n_Z) of n_Z / N
  for (int s = 0; s < 2 * N; ++s) {
    p->row_low.push_back(0);
    p->row_high.push_back(s < N ? n_X : n_Z);
    p->row_cnt.push_back(s < N ? n_X / N : n_Z / N);
  }
  p->shipped_ev.resize(nbuf, nullptr);
  for (int k = 0; k < nbuf; ++k) {
    // no system-scope fence at the record: the worker only needs the uploads to have run
    // (their reads of the pinned buffer are over), not device writes made visible to the
    // host — and a fenced record costs a cache writeback between two segments on the stream
    if (hipEventCreateWithFlags(&p->shipped_ev[k],
                                hipEventDisableTiming | hipEventDisableSystemFence) !=
        hipSuccess) {
      for (int i = 0; i < k; ++i) (void)hipEventDestroy(p->shipped_ev[i]);
      delete p;
      tw::set_error("tw_draw_pipe_start: hipEventCreate failed");
      return TW_ERR_HIP;
    }
  }
  p->worker = std::thread([p] { p->run(); });
  *out_handle = p;
  return TW_OK;
}

// Block until segment j is in buffer j % nbuf (the caller holds no interpreter lock: ctypes
// releases it).  TW_ERR_ARG / TW_ERR_HIP when the worker stopped on a failing draw or sync.
extern "C" int tw_draw_pipe_wait(void* h, int32_t j) {
  auto* p = (tw::DrawPipe*)h;
  TW_ARG_CHECK(p && j >= 0 && j < (int32_t)p->steps.size(), "tw_draw_pipe_wait: bad segment");
  std::unique_lock<std::mutex> lk(p->mu);
  p->cv.wait(lk, [&] { return p->drawn > j || p->cancel; });
  if (p->drawn > j) return TW_OK;
  tw::set_error("tw_draw_pipe_wait: the draw worker stopped (status %d)", p->rc);
  return p->rc ? p->rc : TW_ERR_ARG;
}

// Segment j's upload (every kernel reading its pinned buffers) has been enqueued on `stream`:
// record it; the worker refills the buffers once it has run.  Segments in order.
extern "C" int tw_draw_pipe_shipped(void* h, int32_t j, void* stream) {
  auto* p = (tw::DrawPipe*)h;
  TW_ARG_CHECK(p && j >= 0 && j < (int32_t)p->steps.size(), "tw_draw_pipe_shipped: bad segment");
  TW_HIP_CHECK(hipEventRecord(p->shipped_ev[j % p->nbuf], (hipStream_t)stream));
  {
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->shipped < j + 1) p->shipped = j + 1;
  }
  p->cv.notify_all();
  return TW_OK;
}

// Stop (a loop that ended early cancels the segments not yet drawn), join, free.  The MT19937
// state is where the last segment drawn left it.
extern "C" int tw_draw_pipe_stop(void* h) {
  auto* p = (tw::DrawPipe*)h;
  if (!p) return TW_OK;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    p->cancel = true;
  }
  p->cv.notify_all();
  if (p->worker.joinable()) p->worker.join();
  for (hipEvent_t e : p->shipped_ev) (void)hipEventDestroy(e);
  delete p;
  return TW_OK;
}
