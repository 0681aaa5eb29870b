// Round 6 probe: does RCCL's ncclCommInitRankConfig with blocking = 0 return
// ncclInProgress at once (the NCCL-documented non-blocking set-up), bare or inside an
// explicit ncclGroupStart/End, when the other rank never arrives?  And does the
// documented abort (ncclCommAbort while in progress) then unwind it?
// usage: nb_init_probe <mode: bare|group>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>
#include <chrono>
#include <thread>
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main(int argc, char **argv) {
  const bool group = argc > 1 && !strcmp(argv[1], "group");
  hipSetDevice(0);
  ncclUniqueId id;
  ncclGetUniqueId(&id);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  const double t0 = now();
  if (group) ncclGroupStart();
  ncclResult_t r = ncclCommInitRankConfig(&comm, 2, id, 0, &cfg);
  printf("[%.2f] init call returned %d (%s)\n", now() - t0, (int)r, ncclGetErrorString(r));
  fflush(stdout);
  if (group) {
    r = ncclGroupEnd();
    printf("[%.2f] group end returned %d\n", now() - t0, (int)r);
    fflush(stdout);
  }
  ncclResult_t a = ncclInProgress;
  while (now() - t0 < 4.0) {
    ncclCommGetAsyncError(comm, &a);
    if (a != ncclInProgress) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  printf("[%.2f] async state %d\n", now() - t0, (int)a);
  fflush(stdout);
  r = ncclCommAbort(comm);
  printf("[%.2f] abort returned %d\n", now() - t0, (int)r);
  fflush(stdout);
  return 0;
}
