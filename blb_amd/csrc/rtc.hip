// rtc.hip -- decode networks compiled at run time with hipRTC (see rtc.hpp).
#include "rtc.hpp"

#include <hip/hiprtc.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <unistd.h>

#include "gf256.hpp"
#include "tuning.hpp"

namespace blbrs {
namespace rtc {
namespace {

// The device headers rs_code.hpp needs, embedded at build time (Makefile: _build/rtc_headers.inc
// wraps each file in a raw string), so the library compiles against exactly the source it was
// built from and needs no file next to it.
struct Header {
    const char* name;
    const char* src;
};
const Header kHeaders[] = {
#include "rtc_headers.inc"
};

constexpr int kMaxK = 16;      // inputs a run-time network takes (planes: 8 VGPRs per input)
constexpr int kMaxNetRows = 8;  // = kMaxRows
constexpr size_t kMaxEntries = 512;  // kernels kept per process; past it, passes stay on tables

// --- network generation --------------------------------------------------------------------

// Output plane (r, p) = XOR of input planes (c, q) with bit p of coef[r][c] * 2^q set
// (multiplying by a constant is GF(2)-linear), emitted as a chain of v_bitop3 XOR3s.  No explicit
// shared temporaries: LLVM's reassociation already shares terms between output planes (the static
// VALU count is the same with Paar-style pair sharing), and long-lived temporaries took RS(12,5)'s
// recovery kernel from 156 VGPRs to 252-280 and 7-35 % slower launches (round 4,
// profiles/r04/rtc_ab; the variant is no longer built).
using Planes = std::vector<std::vector<int>>;  // per output plane, its input signals c * 8 + q

Planes plane_terms(int k, int rows, const uint8_t* coef) {
    const GF& g = gf();
    Planes outs(static_cast<size_t>(rows) * 8);
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < k; ++c)
            for (int q = 0; q < 8; ++q) {
                const uint8_t col = g.mul(coef[r * k + c], static_cast<uint8_t>(1u << q));
                for (int p = 0; p < 8; ++p)
                    if ((col >> p) & 1u) outs[r * 8 + p].push_back(c * 8 + q);
            }
    return outs;
}

int xor_ops(const Planes& outs) {
    int n = 0;
    for (const auto& o : outs) n += o.size() <= 1 ? 0 : static_cast<int>(o.size()) / 2;
    return n;
}

std::string sig_name(int s) { return "x[" + std::to_string(s / 8) + "][" + std::to_string(s % 8) + "]"; }

// One output plane: its signals folded by XOR3s.
std::string fold_expr(const std::vector<int>& s) {
    if (s.empty()) return "0u";
    if (s.size() == 1) return sig_name(s[0]);
    if (s.size() == 2) return sig_name(s[0]) + " ^ " + sig_name(s[1]);
    std::string e = "xor3(" + sig_name(s[0]) + ", " + sig_name(s[1]) + ", " + sig_name(s[2]) + ")";
    size_t i = 3;
    for (; i + 1 < s.size(); i += 2) e = "xor3(" + e + ", " + sig_name(s[i]) + ", " + sig_name(s[i + 1]) + ")";
    if (i < s.size()) e = "(" + e + " ^ " + sig_name(s[i]) + ")";
    return e;
}

std::string emit(const Planes& outs, int k, int rows) {
    std::string o;
    o += "struct BlbrsNet {\n  template <int MR>\n  __device__ static __forceinline__ void rows(const uint32_t (&x)[" +
         std::to_string(k) + "][8], uint32_t (&o)[MR][8]) {\n";
    o += "    static_assert(MR == " + std::to_string(rows) + ", \"rows\");\n";
    o += "    using blbrs::dev::xor3;\n";
    for (int r = 0; r < rows; ++r)
        for (int p = 0; p < 8; ++p)
            o += "    o[" + std::to_string(r) + "][" + std::to_string(p) + "] = " + fold_expr(outs[r * 8 + p]) + ";\n";
    o += "#pragma unroll\n    for (int r = 0; r < MR; ++r) blbrs::bs::transpose8(o[r]);\n  }\n";
    // each<MR>(x, f): the same rows one at a time, f(r, row) as soon as row r is in byte form.
    o += "  template <int MR, class F>\n  __device__ static __forceinline__ void each(const uint32_t (&x)[" + std::to_string(k) +
         "][8], F& f) {\n    static_assert(MR == " + std::to_string(rows) + ", \"rows\");\n    using blbrs::dev::xor3;\n";
    for (int r = 0; r < rows; ++r) {
        o += "    {\n      uint32_t o[8];\n";
        for (int p = 0; p < 8; ++p) o += "      o[" + std::to_string(p) + "] = " + fold_expr(outs[r * 8 + p]) + ";\n";
        o += "      blbrs::bs::transpose8(o);\n      f(" + std::to_string(r) + ", o);\n    }\n";
    }
    o += "  }\n};\n";
    return o;
}

// --- state ---------------------------------------------------------------------------------

struct Compiled {
    std::vector<char> code;
    std::string lowered;
};

struct Job {
    std::string src, name_expr;
    int device = 0;
    NetKernel* nk = nullptr;
};

struct State {
    std::mutex mu;
    std::condition_variable cv_idle;
    std::condition_variable cv_work;  // the worker waits here for jobs (or exit)
    std::map<std::string, std::unique_ptr<NetKernel>> kernels;        // device|source
    std::map<std::string, std::shared_ptr<Compiled>> compiled;        // source
    std::deque<Job> queue;
    // Started by the first queued job, joined at exit.  Owned by the process that started it: a
    // fork()ed child inherits the object but not the thread, so it starts (and joins) its own.
    std::thread* worker = nullptr;
    pid_t worker_pid = 0;
    int busy = 0;
    bool exiting = false;
    Stats st;
    std::string first_failure;
};
State& S() {
    static State* s = new State;  // never destroyed: a worker may outlive static destructors
    return *s;
}

void note_failure(State& s, const std::string& what) {
    ++s.st.failed;
    if (s.first_failure.empty()) {
        s.first_failure = what;
        std::fprintf(stderr, "blbrs: run-time decode network unavailable, tables used instead: %.400s\n", what.c_str());
    }
}

void exit_hook_again();

// Everything this module does through comgr (LLVM in this process) -- a hipRTC compile, a
// hipModuleLoadData -- holds this lock, so no two of them overlap: compiles on the worker and
// module loads on launching threads did overlap, and such runs ended in LLVM errors inside
// hiprtcCompileProgram and heap corruption (tools/comgr_race.py).
std::mutex& comgr_mu() {
    static std::mutex* m = new std::mutex;
    return *m;
}

// hipRTC, opened on first use (dlopen), not linked: a process that never asks for a run-time
// network (no RS(12,5)-wide multi-row pass, or BLBRS_RTC = 0) never maps hipRTC or the LLVM
// (comgr) it loads.
struct Hiprtc {
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcAddNameExpression) add_name = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) log = nullptr;
    decltype(&hiprtcGetErrorString) error_string = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) code = nullptr;
    decltype(&hiprtcGetLoweredName) lowered_name = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    std::string error;  // why it is unavailable ("" when loaded)
};

template <class F>
bool sym(void* h, const char* name, F* out, std::string* err) {
    *out = reinterpret_cast<F>(dlsym(h, name));
    if (!*out && err->empty()) *err = std::string("hipRTC: no symbol ") + name;
    return *out != nullptr;
}

const Hiprtc& hiprtc() {
    static const Hiprtc* api = [] {
        auto* a = new Hiprtc;  // process lifetime, as the library handle
        void* h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libhiprtc.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            a->error = std::string("hipRTC not loadable: ") + (e ? e : "dlopen failed");
            return a;
        }
        std::string err;
        int ok = 1;  // every symbol is looked up, so the error names the first missing one
        ok &= sym(h, "hiprtcCreateProgram", &a->create, &err);
        ok &= sym(h, "hiprtcAddNameExpression", &a->add_name, &err);
        ok &= sym(h, "hiprtcCompileProgram", &a->compile, &err);
        ok &= sym(h, "hiprtcGetProgramLogSize", &a->log_size, &err);
        ok &= sym(h, "hiprtcGetProgramLog", &a->log, &err);
        ok &= sym(h, "hiprtcGetErrorString", &a->error_string, &err);
        ok &= sym(h, "hiprtcGetCodeSize", &a->code_size, &err);
        ok &= sym(h, "hiprtcGetCode", &a->code, &err);
        ok &= sym(h, "hiprtcGetLoweredName", &a->lowered_name, &err);
        ok &= sym(h, "hiprtcDestroyProgram", &a->destroy, &err);
        if (!ok) a->error = err;
        return a;
    }();
    return *api;
}

// Compile (outside the state lock); nullptr + log on failure.
std::shared_ptr<Compiled> compile(const std::string& src, const std::string& name_expr, std::string* log) {
    const Hiprtc& rt = hiprtc();
    if (!rt.error.empty()) {
        *log = rt.error;
        return nullptr;
    }
    std::lock_guard<std::mutex> comgr(comgr_mu());
    std::vector<const char*> names, srcs;
    for (const Header& h : kHeaders) {
        names.push_back(h.name);
        srcs.push_back(h.src);
    }
    hiprtcProgram prog = nullptr;
    if (rt.create(&prog, src.c_str(), "blbrs_net.hip", static_cast<int>(names.size()), srcs.data(), names.data()) !=
        HIPRTC_SUCCESS) {
        *log = "hiprtcCreateProgram failed";
        return nullptr;
    }
    rt.add_name(prog, name_expr.c_str());
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult rc = rt.compile(prog, 3, opts);
    std::shared_ptr<Compiled> out;
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        rt.log_size(prog, &n);
        std::string l(n, '\0');
        if (n) rt.log(prog, &l[0]);
        *log = std::string(rt.error_string(rc)) + ": " + l;
    } else {
        out = std::make_shared<Compiled>();
        size_t n = 0;
        rt.code_size(prog, &n);
        out->code.resize(n);
        rt.code(prog, out->code.data());
        const char* lowered = nullptr;
        if (rt.lowered_name(prog, name_expr.c_str(), &lowered) != HIPRTC_SUCCESS || !lowered) {
            *log = "hiprtcGetLoweredName failed for " + name_expr;
            out.reset();
        } else {
            out->lowered = lowered;
        }
    }
    rt.destroy(&prog);
    exit_hook_again();
    return out;
}

// Compile if needed and publish the code object (state 2); ready() loads it.  No HIP call.
void run_job(State& s, const Job& j) {
    std::shared_ptr<Compiled> c;
    {
        std::lock_guard<std::mutex> g(s.mu);
        auto it = s.compiled.find(j.src);
        if (it != s.compiled.end()) c = it->second;
    }
    if (!c) {
        std::string log;
        const auto t0 = std::chrono::steady_clock::now();
        c = compile(j.src, j.name_expr, &log);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::lock_guard<std::mutex> g(s.mu);
        s.st.compile_ms += ms;
        if (!c) {
            note_failure(s, log);
            j.nk->state.store(-1);
            return;
        }
        ++s.st.compiled;
        s.compiled[j.src] = c;   // entries are never erased: `c` outlives every NetKernel
    }
    j.nk->code.store(c.get(), std::memory_order_release);
    j.nk->state.store(2, std::memory_order_release);
}

// Load a compiled code object on nk->device in this thread (comgr_mu held).
void load(State& s, NetKernel* nk) {
    const Compiled* c = static_cast<const Compiled*>(nk->code.load(std::memory_order_acquire));
    int prev = 0;
    (void)hipGetDevice(&prev);
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    hipError_t e = hipSetDevice(nk->device);
    if (e == hipSuccess) e = hipModuleLoadData(&mod, c->code.data());
    if (e == hipSuccess) e = hipModuleGetFunction(&fn, mod, c->lowered.c_str());
    (void)hipSetDevice(prev);
    exit_hook_again();
    std::lock_guard<std::mutex> g(s.mu);
    if (e != hipSuccess || !fn) {
        (void)hipGetLastError();
        note_failure(s, std::string("module load: ") + hipGetErrorString(e));
        nk->state.store(-1);
        return;
    }
    ++s.st.loaded;
    nk->fn.store(fn, std::memory_order_release);
    nk->state.store(1, std::memory_order_release);
}

// One compiler thread for the life of the process: it sleeps on cv_work while idle and ends
// only at exit, where at_exit joins it, so its thread-local teardown (LLVM's, inside hipRTC) is
// over before the process's static destructors run.
void worker_loop() {
    State& s = S();
    std::unique_lock<std::mutex> lk(s.mu);
    for (;;) {
        s.cv_work.wait(lk, [&] { return s.exiting || !s.queue.empty(); });
        if (s.exiting) break;
        Job j = std::move(s.queue.front());
        s.queue.pop_front();
        ++s.busy;
        lk.unlock();
        run_job(s, j);
        lk.lock();
        --s.busy;
        if (s.st.pending) --s.st.pending;
        if (s.queue.empty()) s.cv_idle.notify_all();
    }
    s.cv_idle.notify_all();
}

// At exit: stop taking jobs and let a running compile finish before the compiler is torn down.
// hipRTC runs LLVM (comgr) in this process, and comgr's static destructors run at exit in
// reverse order of registration: a compile still running on the worker when they run aborts the
// process (seen: "LLVM ERROR: Cannot implicitly convert a scalable size ...", and a corrupted
// heap, at the exit of a program whose last calls had queued networks).  So the handler is
// registered after comgr is loaded (exit_hook), again after every compile and module load
// (LLVM's lazily built statics), and it runs before either set of destructors.  It joins the worker
// rather than waiting for a flag, so the thread's own teardown (LLVM thread-locals) is also
// finished before them: a detached worker that ended as exit began crashed there (segfault at
// the exit of tests/cpp/rs_test, 1 run in 2).
void at_exit() {
    State& s = S();
    std::unique_lock<std::mutex> lk(s.mu);
    s.exiting = true;
    s.st.pending -= std::min<uint64_t>(s.st.pending, s.queue.size());
    s.queue.clear();
    s.cv_work.notify_all();
    lk.unlock();
    // Only the library's own worker is waited for: its code after the compile is this file's.
    // A caller thread compiling (BLBRS_RTC = 2, blbrs_rtc_compile) returns into its caller, whose
    // runtime may already be gone (a Python daemon thread crashes there), so it is not held.
    if (s.worker && s.worker_pid == getpid() && s.worker->joinable() &&
        s.worker->get_id() != std::this_thread::get_id())
        s.worker->join();
}

// Loads comgr (hiprtcCreateProgram does; no compile) and then registers at_exit, once.  Called
// before the first compile of the process, without s.mu held.
void exit_hook() {
    static std::once_flag once;
    std::call_once(once, [] {
        const Hiprtc& rt = hiprtc();
        if (rt.error.empty()) {
            std::lock_guard<std::mutex> comgr(comgr_mu());
            hiprtcProgram p = nullptr;
            if (rt.create(&p, "", "blbrs_load.hip", 0, nullptr, nullptr) == HIPRTC_SUCCESS) rt.destroy(&p);
        }
        std::atexit(at_exit);
    });
}

// After every compile and module load: once more, behind whatever statics comgr / LLVM built
// lazily on the way (their destructors then run after at_exit).  Bounded; at_exit is idempotent.
void exit_hook_again() {
    static std::atomic<int> n{0};
    if (n.fetch_add(1, std::memory_order_relaxed) < 4096) std::atexit(at_exit);
}

std::string kernel_source(int k, int rows, const uint8_t* coef, int* ops) {
    const Planes outs = plane_terms(k, rows, coef);
    if (ops) *ops = xor_ops(outs);
    return emit(outs, k, rows);
}

// Handed out once kMaxEntries kernels exist: a pass's slot caches it, so the pass stays on tables
// without generating its source again on every launch.
NetKernel* disabled() {
    static NetKernel* nk = [] {
        auto* p = new NetKernel;
        p->state.store(-1);
        return p;
    }();
    return nk;
}

}  // namespace

// Single-row passes (the client's usual ReconstructData) stay on tables: the network transposes
// all k inputs for one output row and measured 0.2-1 % slower there (profiles/r04/rpc_shapes).
bool eligible(int k, int rows) {
    const long mode = tune::get(tune::kRtc);
    return mode != 0 && k >= 2 && k <= kMaxK && rows >= 2 && rows <= kMaxNetRows &&
           k + rows > tune::get(tune::kRtcWide);
}

std::string network_source(int k, int rows, const uint8_t* coef, int* ops) { return kernel_source(k, rows, coef, ops); }

namespace {
// The translation unit hipRTC compiles for one pass, and the kernel's name expression.
void unit(int k, int rows, Mode mode, bool strided, const uint8_t* coef, std::string* src, std::string* name, int* u,
          int* ops) {
    const int imode = static_cast<int>(mode), addr = strided ? 0 : 1;
    *u = network_u(k, rows, imode);
    *src = "#include \"rs_code.hpp\"\n" + kernel_source(k, rows, coef, ops);
    *name = "blbrs::code::rs_code_kernel<" + std::to_string(k) + ", " + std::to_string(rows) + ", " +
            std::to_string(imode) + ", " + std::to_string(addr) + ", " + std::to_string(*u) + ", 3, BlbrsNet>";
    *src += "// " + *name + "\n";
}
}  // namespace

bool compile_only(int k, int rows, Mode mode, bool strided, const uint8_t* coef, std::string* log,
                  std::vector<char>* code) {
    std::string src, name;
    int u = 0, ops = 0;
    unit(k, rows, mode, strided, coef, &src, &name, &u, &ops);
    State& s = S();
    exit_hook();
    {
        std::lock_guard<std::mutex> g(s.mu);
        auto it = s.compiled.find(src);
        if (it != s.compiled.end()) {
            if (code) *code = it->second->code;
            return true;
        }
        if (s.exiting) {
            *log = "process exiting";
            return false;
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto c = compile(src, name, log);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> g(s.mu);
    s.st.compile_ms += ms;
    if (!c) return false;
    ++s.st.compiled;
    s.compiled[src] = c;
    if (code) *code = c->code;
    return true;
}

NetKernel* request(int device, int k, int rows, Mode mode, bool strided, const uint8_t* coef) {
    if (!eligible(k, rows)) return nullptr;
    State& s = S();
    {
        // Past the cap, before building a source of up to ~30 KB that could not be used anyway.
        std::lock_guard<std::mutex> g(s.mu);
        if (s.kernels.size() >= kMaxEntries) return disabled();
    }
    std::string src, name;
    int u = 0, ops = 0;
    unit(k, rows, mode, strided, coef, &src, &name, &u, &ops);
    const std::string key = std::to_string(device) + "|" + src;
    exit_hook();
    NetKernel* nk = nullptr;
    bool sync = false;
    {
        std::lock_guard<std::mutex> g(s.mu);
        auto it = s.kernels.find(key);
        if (it != s.kernels.end()) return it->second.get();
        if (s.exiting) return nullptr;
        if (s.kernels.size() >= kMaxEntries) return disabled();
        auto p = std::make_unique<NetKernel>();
        p->device = device;
        p->u = u;
        p->ops = ops;
        nk = p.get();
        s.kernels.emplace(key, std::move(p));
        ++s.st.requested;
        sync = tune::get(tune::kRtc) == 2;
        if (!sync) {
            s.queue.push_back(Job{src, name, device, nk});
            ++s.st.pending;
            if (!s.worker || s.worker_pid != getpid()) {
                s.worker = new std::thread(worker_loop);  // never deleted: see State
                s.worker_pid = getpid();
            } else {
                s.cv_work.notify_one();
            }
        } else {
            ++s.busy;
        }
    }
    if (sync) {
        run_job(s, Job{src, name, device, nk});
        (void)ready(nk, /*wait=*/true);
        std::lock_guard<std::mutex> g(s.mu);
        --s.busy;
        s.cv_idle.notify_all();
    }
    return nk;
}

hipFunction_t ready(NetKernel* nk, bool wait) {
    if (!nk) return nullptr;
    if (hipFunction_t f = nk->fn.load(std::memory_order_acquire)) return f;
    if (nk->state.load(std::memory_order_acquire) != 2) return nullptr;
    State& s = S();
    // A launch does not wait for a compile in progress: the tables serve it, a later launch loads.
    std::unique_lock<std::mutex> comgr(comgr_mu(), std::defer_lock);
    if (wait) comgr.lock();
    else if (!comgr.try_lock()) return nullptr;
    if (nk->state.load(std::memory_order_acquire) == 2) load(s, nk);
    return nk->fn.load(std::memory_order_acquire);
}

Stats stats() {
    State& s = S();
    std::lock_guard<std::mutex> g(s.mu);
    return s.st;
}

bool wait_idle(long timeout_ms) {
    State& s = S();
    std::unique_lock<std::mutex> lk(s.mu);
    auto idle = [&] { return s.queue.empty() && s.busy == 0; };
    if (timeout_ms < 0) {
        s.cv_idle.wait(lk, idle);
        return true;
    }
    return s.cv_idle.wait_for(lk, std::chrono::milliseconds(timeout_ms), idle);
}

std::string first_failure() {
    State& s = S();
    std::lock_guard<std::mutex> g(s.mu);
    return s.first_failure;
}

}  // namespace rtc
}  // namespace blbrs
