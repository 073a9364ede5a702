// Test stub standing in for librccl (tests/test_comm_failure.py): the handful of RCCL entry
// points csrc/comm.hip binds, with ncclCommGetAsyncError reporting a peer failure
// (STUB_MODE=error), a collective that never finishes (STUB_MODE=inprogress) or nothing wrong
// (STUB_MODE=ok: the GPU test of a slow count queued before the collective), so the
// failure-detection path of tw_comm_wait runs without peers.
#include <cstdlib>
#include <cstring>

extern "C" {
typedef struct ncclComm* ncclComm_t;
static int g_aborts = 0, g_gathers = 0;
static int mode() {
  const char* m = std::getenv("STUB_MODE");
  if (m && std::strcmp(m, "ok") == 0) return 0;
  return (m && std::strcmp(m, "inprogress") == 0) ? 7 : 2;  // ncclInProgress / ncclSystemError
}
int ncclCommInitAll(ncclComm_t* comms, int n, const int*) {
  for (int i = 0; i < n; ++i) comms[i] = (ncclComm_t)(std::size_t)(0x1000 + i);
  return 0;
}
int ncclCommDestroy(ncclComm_t) { return 0; }
int ncclCommAbort(ncclComm_t) { ++g_aborts; return 0; }
int ncclAllGather(const void*, void*, std::size_t, int, ncclComm_t, void*) {
  ++g_gathers;
  return 0;
}
int ncclGroupStart() { return 0; }
int ncclGroupEnd() { return 0; }
const char* ncclGetErrorString(int e) { return e == 2 ? "stub: system error" : "stub: other"; }
int ncclCommGetAsyncError(ncclComm_t, int* err) {
  *err = mode();
  return 0;
}
int stub_aborts() { return g_aborts; }
int stub_gathers() { return g_gathers; }
}
