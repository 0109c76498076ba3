// phd_crash.cpp -- crash triage for the library's callers (bench.py's
// PHD_BENCH_MAPS): a fault's raw return addresses only resolve to library +
// offset against the mappings of the process AT the fault, so the handler
// writes /proc/self/maps then, not at some earlier point of the run.  Only
// async-signal-safe calls (open / read / write / close / getpid / sigaction /
// raise) run in the handler; the previous handler (a profiler's or a
// runtime's stack printer) still runs afterwards.
#include <csignal>
#include <cstring>

#include <fcntl.h>
#include <unistd.h>

#include "../../include/photohive_dsp.h"

namespace {

constexpr int kSigs[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
constexpr int kNSig = sizeof(kSigs) / sizeof(kSigs[0]);
struct sigaction g_prev[kNSig];
char g_prefix[512];
volatile sig_atomic_t g_busy = 0;

size_t put_str(char* d, size_t o, size_t cap, const char* s) {
    while (*s && o + 1 < cap) d[o++] = *s++;
    return o;
}
size_t put_uint(char* d, size_t o, size_t cap, unsigned long v) {
    char t[24];
    int n = 0;
    do {
        t[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v && n < 24);
    while (n && o + 1 < cap) d[o++] = t[--n];
    return o;
}

void write_maps() {
    char path[600];
    size_t o = put_str(path, 0, sizeof(path), g_prefix);
    o = put_str(path, o, sizeof(path), ".");
    o = put_uint(path, o, sizeof(path), (unsigned long)getpid());
    o = put_str(path, o, sizeof(path), ".maps");
    path[o] = 0;
    const int in = open("/proc/self/maps", O_RDONLY);
    if (in < 0) return;
    const int out = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (out >= 0) {
        char buf[4096];
        for (ssize_t k; (k = read(in, buf, sizeof(buf))) > 0;)
            if (write(out, buf, (size_t)k) != k) break;
        close(out);
    }
    close(in);
}

void on_fault(int sig, siginfo_t* info, void* uc) {
    if (!g_busy) {
        g_busy = 1;
        write_maps();
    }
    for (int i = 0; i < kNSig; i++) {
        if (kSigs[i] != sig) continue;
        const struct sigaction& p = g_prev[i];
        if (p.sa_flags & SA_SIGINFO) {
            if (p.sa_sigaction) {
                p.sa_sigaction(sig, info, uc);
                return;
            }
        } else if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
            p.sa_handler(sig);
            return;
        }
        // default action: restore it and re-raise (a fault re-executes and
        // faults again under the default disposition)
        struct sigaction d;
        memset(&d, 0, sizeof(d));
        d.sa_handler = SIG_DFL;
        sigemptyset(&d.sa_mask);
        sigaction(sig, &d, nullptr);
        raise(sig);
        return;
    }
}

}  // namespace

extern "C" int phd_install_crash_maps(const char* prefix) {
    if (!prefix || !*prefix || strlen(prefix) >= sizeof(g_prefix)) return -1;
    memcpy(g_prefix, prefix, strlen(prefix) + 1);
    for (int i = 0; i < kNSig; i++) {
        struct sigaction a;
        memset(&a, 0, sizeof(a));
        a.sa_sigaction = on_fault;
        a.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigemptyset(&a.sa_mask);
        if (sigaction(kSigs[i], &a, &g_prev[i]) != 0) return -1;
    }
    return 0;
}
