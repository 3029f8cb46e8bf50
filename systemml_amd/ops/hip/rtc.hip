// Run-time compilation of generated kernels (reference: hops/codegen/SpoofCompiler.java
// compiles each generated operator class with janino / javac at run time and caches it by
// its source; SystemML's later GPU codegen does the same with NVRTC).
//
// Here the generated source (ops/cell.py#generate: a `Spec` struct + the device templates of
// ops/hip/cell_rtc.inc) is compiled by hipRTC for the device's gfx target into a code object,
// which the caller caches in memory and on disk by the source's hash and loads with
// hipModuleLoadData.  Launches pass the kernel's single by-value argument struct through the
// HIP_LAUNCH_PARAM_BUFFER_POINTER interface on the caller's (PyTorch's current) stream.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <string.h>

extern "C" {

// Compile `src` for `arch` (e.g. "gfx950").  On success returns 0 and the code object size in
// *size; the bytes are then fetched with sysml_rtc_code (same handle).  On failure returns the
// hiprtc error code (> 0) and copies the compiler log into log[0:loglen].
int sysml_rtc_compile(const char* src, const char* name, const char* arch, void** handle, size_t* size, char* log,
                      size_t loglen) {
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, src, name, 0, nullptr, nullptr);
  if (r != HIPRTC_SUCCESS) return (int)r;
  char archopt[64];
  snprintf(archopt, sizeof(archopt), "--offload-arch=%s", arch);
  const char* opts[] = {archopt, "-O3", "-ffp-contract=off", "-std=c++17"};
  r = hiprtcCompileProgram(prog, 4, opts);
  if (r != HIPRTC_SUCCESS) {
    size_t ls = 0;
    if (log && loglen && hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 0) {
      char* buf = new char[ls + 1];
      hiprtcGetProgramLog(prog, buf);
      buf[ls] = 0;
      strncpy(log, buf, loglen - 1);
      log[loglen - 1] = 0;
      delete[] buf;
    }
    hiprtcDestroyProgram(&prog);
    return (int)r;
  }
  r = hiprtcGetCodeSize(prog, size);
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return (int)r;
  }
  hiprtcProgram* h = new hiprtcProgram(prog);
  *handle = h;
  return 0;
}

// Copy the compiled code object into `code` (size from sysml_rtc_compile) and release the program.
int sysml_rtc_code(void* handle, void* code) {
  hiprtcProgram* h = static_cast<hiprtcProgram*>(handle);
  hiprtcResult r = hiprtcGetCode(*h, static_cast<char*>(code));
  hiprtcDestroyProgram(h);
  delete h;
  return (int)r;
}

// Load a code object and look up kernel `name`; the module stays loaded for the process.
int sysml_rtc_load(const void* code, const char* name, void** func) {
  hipModule_t mod;
  hipError_t e = hipModuleLoadData(&mod, code);
  if (e != hipSuccess) return (int)e;
  hipFunction_t f;
  e = hipModuleGetFunction(&f, mod, name);
  if (e != hipSuccess) return (int)e;
  *func = (void*)f;
  return 0;
}

int sysml_rtc_launch(void* func, unsigned gx, unsigned gy, unsigned bx, void* args, size_t args_size,
                     void* stream) {
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &args_size,
                 HIP_LAUNCH_PARAM_END};
  hipError_t e = hipModuleLaunchKernel((hipFunction_t)func, gx, gy, 1, bx, 1, 1, 0,
                                       reinterpret_cast<hipStream_t>(stream), nullptr, cfg);
  return (int)e;
}

}  // extern "C"
