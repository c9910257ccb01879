/* Diagnostic only (never linked into the library): a native crash reporter loaded into a test process
 * with ctypes.CDLL when FVHIP_CRASHTRACE is set (tests/rccl_rank_worker.py). On SIGSEGV / SIGBUS /
 * SIGILL / SIGFPE / SIGABRT it writes to stderr the signal, the faulting address, the thread that
 * faulted (kernel tid and name: the main thread or a runtime/RCCL helper thread), the native
 * backtrace (libraries + offsets, resolvable offline with addr2line against the same .so files), and
 * the mapped libraries, then re-raises with the default action.
 * build: gcc -shared -fPIC -O1 -g -o tools/bin/libcrashtrace.so tools/probes/crashtrace.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <fcntl.h>

static char altstack[1 << 16];

static void say(const char* s) { ssize_t r = write(2, s, strlen(s)); (void)r; }

static void handler(int sig, siginfo_t* si, void* ctx) {
	(void)ctx;
	char buf[512], name[32] = {0};
	prctl(PR_GET_NAME, name, 0, 0, 0);
	snprintf(buf, sizeof buf, "\n=== crashtrace: signal %d (code %d) at address %p, tid %ld ('%s'), pid %d ===\n",
	         sig, si ? si->si_code : 0, si ? si->si_addr : 0, (long)syscall(SYS_gettid), name, (int)getpid());
	say(buf);
	void* fr[64];
	const int n = backtrace(fr, 64);
	backtrace_symbols_fd(fr, n, 2);
	say("=== crashtrace: mapped executable regions ===\n");
	const int fd = open("/proc/self/maps", O_RDONLY);
	if(fd >= 0) {
		char line[4096];
		ssize_t k;
		size_t used = 0;
		/* copy lines holding "r-xp" (code) to stderr */
		while((k = read(fd, line + used, sizeof line - 1 - used)) > 0) {
			used += (size_t)k;
			line[used] = 0;
			char* s = line;
			char* nl;
			while((nl = strchr(s, '\n'))) {
				*nl = 0;
				if(strstr(s, "r-xp") && strchr(s, '/')) { say(s); say("\n"); }
				s = nl + 1;
			}
			used = strlen(s);
			memmove(line, s, used);
		}
		close(fd);
	}
	say("=== crashtrace: end ===\n");
	signal(sig, SIG_DFL);
	raise(sig);
}

__attribute__((constructor)) static void install(void) {
	stack_t ss;
	ss.ss_sp = altstack;
	ss.ss_size = sizeof altstack;
	ss.ss_flags = 0;
	sigaltstack(&ss, 0);
	struct sigaction sa;
	memset(&sa, 0, sizeof sa);
	sa.sa_sigaction = handler;
	sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_RESETHAND;
	sigemptyset(&sa.sa_mask);
	const int sigs[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
	for(size_t i = 0; i < sizeof sigs/sizeof sigs[0]; i++) sigaction(sigs[i], &sa, 0);
}
