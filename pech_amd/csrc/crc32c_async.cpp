// crc32c_async.cpp -- the messenger-facing layer (include/pech_crc32c_async.h):
// pinned payload pages, eventfd-completed payload batches, concatenation.
//
// Data path of one async context (up to four staging slots in flight, each
// with its own HIP stream and workspace, so small batches overlap):
//   submit()   places the payload in the slot being filled -- pageable bytes
//              are packed into the slot's pinned staging buffer (one CPU
//              copy, one H2D per slot); crc32c_pages payloads are read by
//              the kernel in place over the host link (the default), or,
//              with CRC32C_ASYNC_DMA, packed below 32 KiB and DMA'd from
//              where they lie above (copies recorded here, issued at the
//              slot's launch) -- and records one descriptor per piece.
//              A payload larger than what a slot has left is cut into
//              pieces; piece 0 carries the seed, later pieces seed 0.
//   flush()    DMA of the recorded payloads and H2D of the packed staging
//              runs, plan + main kernels (the plan reads the descriptors in
//              place from pinned memory), D2H of the results, and a host
//              function that marks the slot finished and bumps the eventfd
//              -- four stream operations per batch.
//   complete() harvests finished slots in launch order, folds each piece
//              into its payload (crc <- crc32c_combine(crc, piece, len)),
//              frees the slot, and runs the callbacks of finished payloads
//              in submission order on the caller's thread.
// No byte is checksummed on the CPU: pieces and combine are GF(2) algebra
// on kernel results (gf2.h).
// Every HIP call runs on the library stack (on_lib_stack, crc32c_cpu.c);
// callbacks run on the caller's own stack, outside the device guard, so a
// callback may switch coroutines or submit again.
// Failures: a failed H2D, launch or batch fails every payload with a piece
// in that slot (callback err = -EIO), makes the context's error sticky and
// bumps the eventfd so the loop collects them.  A submission that returns
// an error never gets a callback -- also when its own submit filled the slot
// and that launch failed.  A batch that fails after its launch (the stream
// reports an error, so its host function never runs and the eventfd stays
// quiet) is found by the next complete() or drain(), which ask the stream:
// an epoll loop calls complete() when the fd fires AND from a timer while
// crc32c_async_pending() > 0 (include/pech_crc32c_async.h).
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <linux/futex.h>
#include <stdlib.h>
#include <sys/syscall.h>
#include <time.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <thread>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/pech_crc32c_async.h"
#include "api_internal.h"
#include "gf2.h"
#include "layout.h"

#define TRY_HIP(expr, ret)                                                                              \
	do {                                                                                            \
		hipError_t e_ = (expr);                                                                 \
		if (e_ != hipSuccess) {                                                                 \
			pech_internal_set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
					      __LINE__);                                                \
			return ret;                                                                     \
		}                                                                                       \
	} while (0)

// ===========================================================================
// pinned payload pages (src/page.c:73-146 semantics, pinned + GPU-mapped)
namespace {

struct PageAlloc {
	size_t bytes;
	void *dev; // device address of the mapping (hipHostGetDevicePointer)
	bool live; // handed out (not on a free list)
};

constexpr unsigned kMaxOrder = CRC32C_PAGES_MAX_ORDER;
constexpr size_t kMaxCachedPerOrder = 32u << 20; // src/page.c:6

std::mutex g_pages_mu;
std::map<uintptr_t, PageAlloc> g_pages;          // every pinned allocation, by base
std::vector<void *> g_free[kMaxOrder + 1];       // cached free allocations per order

// [p, p+len) inside one live allocation: its entry, else end()
std::map<uintptr_t, PageAlloc>::iterator find_live(const void *p, size_t len)
{
	const uintptr_t a = (uintptr_t)p;
	auto it = g_pages.upper_bound(a);
	if (it == g_pages.begin())
		return g_pages.end();
	--it;
	if (!it->second.live || a + len > it->first + it->second.bytes || a + len < a)
		return g_pages.end();
	return it;
}

} // namespace

static void *pages_alloc(unsigned int order)
{
	if (order > 31u - CRC32C_PAGE_SHIFT) {
		pech_internal_set_err("crc32c_pages_alloc: order %u too large", order);
		return nullptr;
	}
	const size_t bytes = (size_t)CRC32C_PAGE_SIZE << order;
	std::lock_guard<std::mutex> lk(g_pages_mu);
	if (order <= kMaxOrder && !g_free[order].empty()) {
		void *p = g_free[order].back();
		g_free[order].pop_back();
		g_pages[(uintptr_t)p].live = true;
		return p;
	}
	void *p = nullptr;
	TRY_HIP(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable), nullptr);
	void *d = nullptr;
	if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d)
		d = p; // unified addressing: the host address is the device address
	g_pages[(uintptr_t)p] = PageAlloc{bytes, d, true};
	return p;
}

extern "C" void *crc32c_pages_alloc(unsigned int order)
{
	void *p = nullptr;
	on_lib_stack([&] {
		p = pages_alloc(order);
		return 0;
	});
	return p;
}

static void pages_free(void *pages, unsigned int order)
{
	std::lock_guard<std::mutex> lk(g_pages_mu);
	auto it = g_pages.find((uintptr_t)pages);
	if (it == g_pages.end() || !it->second.live || it->second.bytes != ((size_t)CRC32C_PAGE_SIZE << order)) {
		fprintf(stderr, "pech_crc32c: crc32c_pages_free(%p, %u): not a live allocation of that order\n", pages,
			order);
		abort(); // a bad free in pech is a BUG_ON (src/page.c keeps no checks)
	}
	if (order <= kMaxOrder && g_free[order].size() < (kMaxCachedPerOrder >> CRC32C_PAGE_SHIFT >> order)) {
		it->second.live = false;
		g_free[order].push_back(pages);
		return;
	}
	g_pages.erase(it);
	(void)hipHostFree(pages);
}

extern "C" void crc32c_pages_free(void *pages, unsigned int order)
{
	if (!pages)
		return;
	on_lib_stack([&] {
		pages_free(pages, order);
		return 0;
	});
}

extern "C" int crc32c_pages_is_pinned(const void *p, size_t len)
{
	std::lock_guard<std::mutex> lk(g_pages_mu);
	return find_live(p, len) != g_pages.end();
}

extern "C" void crc32c_pages_trim(void)
{
	on_lib_stack([] {
		std::lock_guard<std::mutex> lk(g_pages_mu);
		for (auto &fl : g_free) {
			for (void *p : fl) {
				g_pages.erase((uintptr_t)p);
				(void)hipHostFree(p);
			}
			fl.clear();
		}
		return 0;
	});
}

// device address of pinned host bytes p (inside a live allocation), or 0
static uint64_t pinned_dev_addr(const void *p, size_t len)
{
	std::lock_guard<std::mutex> lk(g_pages_mu);
	auto it = find_live(p, len);
	if (it == g_pages.end())
		return 0;
	return (uint64_t)(uintptr_t)it->second.dev + ((uintptr_t)p - it->first);
}

// ===========================================================================
// async contexts
namespace {

// Every entry point that calls HIP runs on its context's device and restores
// the caller's: one thread can drive one context per GPU (SURVEY 7 step 7,
// 8e) without tracking the current device itself.  Lazy: the common submit
// (a descriptor into the open slot) and complete (slots already finished)
// make no HIP call at all, and a HIP call costs the caller's thread more than
// the descriptor does (tools/c/launch_cost.c).
struct DeviceGuard {
	int dev, prev = -1;
	bool tried = false, ok = false, changed = false;
	explicit DeviceGuard(int d, bool now = true) : dev(d)
	{
		if (now)
			ensure();
	}
	bool ensure()
	{
		if (tried)
			return ok;
		tried = true;
		if (hipGetDevice(&prev) != hipSuccess)
			return false;
		changed = prev != dev;
		ok = !changed || hipSetDevice(dev) == hipSuccess;
		return ok;
	}
	~DeviceGuard()
	{
		if (ok && changed)
			(void)hipSetDevice(prev);
	}
};

constexpr size_t kSlotBytes = 32u << 20; // staging per slot
// Zero-copy (the default since round 4) reads every pinned payload in place.
// Until round 3 payloads from 1 MiB up were DMA'd even then: a little more
// link bandwidth (42-50 against 36-37 GiB/s), but 5-40 us of the caller's
// CPU per payload against 0.6 (profiles/r03/ab_zc_max.txt); pech's one
// thread is the budget.
constexpr size_t kZeroCopyMax = SIZE_MAX;
// DMA mode: pinned payloads below this are packed into the slot's staging by
// memcpy (one H2D per slot) instead of one hipMemcpyAsync each: a DMA call
// costs the caller microseconds of CPU, a 4 KiB memcpy a fraction of one
constexpr size_t kDmaMin = 32u << 10;
constexpr uint32_t kSlotDescs = 8192;    // descriptors per slot
// slots whose pieces are all shorter take the direct kernel (one launch, no
// plan): the balanced range of crc32c_dev_batch_small_async
constexpr uint32_t kDirectMax = 32u << 10;
constexpr unsigned kMaxSlots = 4;        // slots in flight per context
constexpr uint64_t kQueryAfterNs = 1000000; // complete(): a stream is queried once its batch is this old
constexpr size_t kPollMax = 8u << 20;       // a lone batch of at most this many bytes is polled (notify)

struct Piece {
	uint64_t item; // submission id
	uint32_t len;
};

// CRC32C_ASYNC_DMA: a payload copy recorded at submit, issued at launch
struct DmaCopy {
	void *dst;
	void *src;
	size_t bytes;
};

// hipMemcpyBatchAsync (HIP 7.1+): one call for a slot's copies.  Resolved at
// run time: a process may have loaded an older HIP runtime first (PyTorch
// bundles its own), and the library must still load there.
typedef hipError_t (*batch_copy_fn)(void **, void **, size_t *, size_t, hipMemcpyAttributes *, size_t *, size_t,
				   size_t *, hipStream_t);
static batch_copy_fn batch_copy()
{
	static const batch_copy_fn f = [] {
		const char *e = getenv("PECH_ASYNC_DMA_BATCH"); // =0: one call per copy (A/B)
		return e && e[0] == '0' ? nullptr : (batch_copy_fn)dlsym(RTLD_DEFAULT, "hipMemcpyBatchAsync");
	}();
	return f;
}

struct Slot {
	hipStream_t stream = nullptr; // own stream and workspace: up to kMaxSlots batches overlap
	void *d_ws = nullptr;
	uint8_t *h_stage = nullptr, *d_stage = nullptr;
	pech_desc *h_desc = nullptr, *d_desc = nullptr;
	const pech_desc *desc_view = nullptr; // device mapping of h_desc: the plan kernel reads it in place
	uint32_t *h_out = nullptr, *d_out = nullptr;
	uint32_t *out_view = nullptr; // device mapping of h_out: flat and direct launches store the results there
	// a flat launch's status word (coherent pinned; layout.h PECH_FLAT_PUB /
	// PECH_FLAT_ERR): checked before the results are taken (slot_verify)
	uint64_t *h_stat = nullptr, *stat_view = nullptr;
	uint64_t flat_tag = 0;  // the slot's flat launch (0: none)
	bool published = false; // ... which stores the results in h_out itself
	std::atomic<int> finished{0}; // set by the stream's host function after the results' D2H
	std::atomic<int> waiting{0};  // a submit sleeps on `finished` (futex): the host function wakes it
	int efd = -1;                 // the context's eventfd
	std::vector<Piece> pieces;
	std::vector<std::pair<size_t, size_t>> packed; // staging runs filled by memcpy: [lo, hi)
	std::vector<DmaCopy> dma;                      // CRC32C_ASYNC_DMA payload copies, issued at launch
	size_t used = 0;     // staging bytes
	size_t zc_bytes = 0; // bytes read in place: a slot launches at kSlotBytes of either
	uint32_t maxlen = 0; // longest piece: the direct kernel takes slots of pieces below kDirectMax
	bool inflight = false;
	bool queued = false;      // CRC32C_ASYNC_DMA: filled, launched once the slots before it are harvested
	bool inject_fail = false; // test build: this batch's stream "failed" (PECH_FAULT_ASYNC_STREAM)
	hipEvent_t ev_done = nullptr; // notifier: recorded after the results' D2H
	uint64_t est_ns = 0;          // notifier: the batch's expected time (host link rate)
	uint64_t t_launch = 0;    // mono_ns() at launch
};

static inline uint64_t mono_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

struct Item {
	crc32c_done_fn done;
	void *arg;
	uint32_t crc;       // folded result of the harvested pieces
	uint32_t harvested; // pieces whose results are folded in
	uint32_t total;     // pieces placed (valid once `placed`)
	bool placed;        // every piece has been given a descriptor
	int err;
	bool cancelled;     // its submit returned an error: no callback
};

} // namespace

struct crc32c_async {
	int dev = -1;
	unsigned flags = 0;
	int efd = -1;
	bool ready = false; // fully created (destroy drains only then)
	bool planned_only = false; // PECH_ASYNC_PLANNED=1: every slot on plan + main (A/B measurement)
	size_t zc_max = kZeroCopyMax; // PECH_ASYNC_ZC_MAX=<bytes>: zero-copy threshold (A/B measurement)
	unsigned max_slots = kMaxSlots; // PECH_ASYNC_SLOTS=<1..4>: slots in flight (A/B measurement)
	std::vector<Slot *> slots;
	std::deque<Slot *> inflight; // launch order
	Slot *cur = nullptr;         // slot being filled
	std::deque<Item> items;      // items[k] is submission id base + k
	uint64_t base = 0;
	int err = 0;                 // sticky failure of this context
	// PECH_ASYNC_PROF=1: the calling thread's CPU ns per phase, printed by
	// destroy (where a DMA-mode thread's time goes; measurement only)
	bool prof = false;
	uint64_t prof_ns[5] = {0, 0, 0, 0, 0}; // copies issued, kernels + D2H + host function, waits for a slot, submit, complete
	uint64_t launches = 0;  // batches launched (crc32c_async_get_stats)
	uint64_t submitted = 0; // submissions accepted
	uint64_t host_out = 0;  // launches whose results the kernel stored in h_out
	uint64_t polled = 0;    // launches notified by the notifier thread
	bool lone_taken = false;  // the messenger adapter host-routed a lone payload since the last flush
	uint64_t faults = 0;      // flat launches whose results the kernel voided (their payloads failed, -EIO)
	uint64_t pub_missing = 0; // flat launches whose in-kernel publication was missing (results copied instead)
	// How a finished batch reaches the eventfd.  A host function on the
	// slot's stream (hipLaunchHostFunc) sleeps until an interrupt, but the
	// runtime takes ~10 us to run it: a lone 64 KiB payload waited 37.7 us
	// p50 for its CRC, 26.7 with the context's notifier thread polling an
	// event recorded after the results' D2H instead -- which costs that
	// thread the batch's duration in CPU (profiles/r05/msgr_notify.txt).  So
	// (3, the default) a batch launched while no other is in flight, of at
	// most kPollMax bytes, is polled -- after sleeping through most of its
	// expected time -- and any other by a host function.
	// PECH_ASYNC_NOTIFY (A/B): 0 = host functions only; 1 = the notifier
	// blocks in hipEventSynchronize (hipEventBlockingSync; it spun: 100 us
	// of CPU per 4 MiB payload); 2 = it polls every batch.
	int notify = 3;
	std::thread notifier;
	std::mutex nmu;
	std::condition_variable ncv;
	std::deque<Slot *> nq; // launched slots, in launch order
	std::atomic<bool> nstop{false};
};

static inline uint64_t thread_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// adds the calling thread's CPU time in its scope to a->prof_ns[k]
struct ProfScope {
	crc32c_async *a;
	int k;
	uint64_t t0;
	ProfScope(crc32c_async *ctx, int kind) : a(ctx->prof ? ctx : nullptr), k(kind), t0(a ? thread_ns() : 0) {}
	void stop()
	{
		if (a)
			a->prof_ns[k] += thread_ns() - t0;
		a = nullptr;
	}
	~ProfScope() { stop(); }
};

static void slot_free(Slot *s)
{
	if (s->stream) {
		(void)hipStreamSynchronize(s->stream);
		(void)hipStreamDestroy(s->stream);
	}
	if (s->d_ws)
		(void)hipFree(s->d_ws);
	if (s->h_stage)
		(void)hipHostFree(s->h_stage);
	if (s->d_stage)
		(void)hipFree(s->d_stage);
	if (s->h_desc)
		(void)hipHostFree(s->h_desc);
	if (s->d_desc)
		(void)hipFree(s->d_desc);
	if (s->h_out)
		(void)hipHostFree(s->h_out);
	if (s->h_stat)
		(void)hipHostFree(s->h_stat);
	if (s->d_out)
		(void)hipFree(s->d_out);
	if (s->ev_done)
		(void)hipEventDestroy(s->ev_done);

	delete s;
}

static Slot *slot_new(int efd)
{
	Slot *s = new Slot();
	if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
	    hipMalloc(&s->d_ws, pech_ws_bytes(kSlotDescs)) != hipSuccess ||
	    hipHostMalloc(&s->h_stage, kSlotBytes, hipHostMallocDefault) != hipSuccess ||
	    hipMalloc(&s->d_stage, kSlotBytes) != hipSuccess ||
	    hipHostMalloc(&s->h_desc, kSlotDescs * sizeof(pech_desc), hipHostMallocDefault) != hipSuccess ||
	    hipMalloc(&s->d_desc, kSlotDescs * sizeof(pech_desc)) != hipSuccess ||
	    hipHostMalloc(&s->h_out, kSlotDescs * 4u, hipHostMallocDefault) != hipSuccess ||
	    hipMalloc(&s->d_out, kSlotDescs * 4u) != hipSuccess ||
	    hipHostMalloc((void **)&s->h_stat, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
		pech_internal_set_err("crc32c_async: slot allocation failed: %s", hipGetErrorString(hipGetLastError()));
		slot_free(s);
		return nullptr;
	}
	s->pieces.reserve(kSlotDescs);
	s->efd = efd;
	void *dv = nullptr;
	if (hipHostGetDevicePointer(&dv, s->h_desc, 0) == hipSuccess && dv)
		s->desc_view = (const pech_desc *)dv;
	else
		(void)hipGetLastError(); // no mapping: descriptors go by H2D copy
	memset(s->h_stat, 0, 64);
	dv = nullptr;
	if (hipHostGetDevicePointer(&dv, s->h_stat, 0) == hipSuccess && dv)
		s->stat_view = (uint64_t *)dv;
	else
		(void)hipGetLastError(); // (no status word: flat launches then take the D2H copy, below)
	const char *ho = getenv("PECH_ASYNC_HOST_OUT"); // A/B: 0 = results by D2H copy after every launch
	dv = nullptr;
	if (!(ho && ho[0] == '0') && s->stat_view && hipHostGetDevicePointer(&dv, s->h_out, 0) == hipSuccess && dv)
		s->out_view = (uint32_t *)dv;
	else
		(void)hipGetLastError();
	return s;
}

// The slot's `finished` flag doubles as a futex word, so a submit that must
// wait for a slot sleeps instead of spinning in hipStreamSynchronize: that
// spin was most of the caller's CPU per payload once the host link is the
// bound (4 MiB payloads: ~140 us of thread CPU each, profiles/r03/msgr_cpu_v17.txt).
static_assert(sizeof(std::atomic<int>) == sizeof(int), "futex word");
static void flag_sleep(std::atomic<int> *f, long ns)
{
	struct timespec ts = {0, ns};
	(void)syscall(SYS_futex, reinterpret_cast<int *>(f), FUTEX_WAIT_PRIVATE, 0, &ts, nullptr, 0);
}

static void host_notify(void *arg)
{
	// HIP runtime thread: only the slot's flags and the eventfd are touched.
	// seq_cst on both sides: either the waiter sees `finished`, or this
	// thread sees `waiting` and wakes it (a wake before its sleep is not
	// lost: the futex wait rechecks the word).
	Slot *s = (Slot *)arg;
	s->finished.store(1, std::memory_order_seq_cst);
	if (s->waiting.load(std::memory_order_seq_cst))
		(void)syscall(SYS_futex, reinterpret_cast<int *>(&s->finished), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr,
			      nullptr, 0);
	const uint64_t one = 1;
	ssize_t r = write(s->efd, &one, sizeof(one));
	(void)r;
}

// fold a harvested slot's results into its items; slot becomes reusable
static void harvest(crc32c_async *a, Slot *s, int err)
{
	for (size_t k = 0; k < s->pieces.size(); ++k) {
		const Piece &pc = s->pieces[k];
		Item &it = a->items[pc.item - a->base];
		if (err)
			it.err = err;
		else
			// pieces arrive in byte order (slots complete in launch order);
			// piece 0 carried the seed, the rest were checksummed from 0
			it.crc = it.harvested == 0 ? s->h_out[k] : crc32c_combine(it.crc, s->h_out[k], pc.len);
		it.harvested++;
	}
	s->pieces.clear();
	s->packed.clear();
	s->dma.clear();
	s->used = 0;
	s->zc_bytes = 0;
	s->maxlen = 0;
	s->inflight = false;
	s->queued = false;
	s->inject_fail = false;
}

static int issue_slot(crc32c_async *a, Slot *s);

// Before a finished slot's results are taken: a flat launch
// reports in its status word whether one of its waves gave up waiting for
// out[]'s initialisation (PECH_FLAT_ERR: the results are void -- the slot's
// payloads fail with -EIO, and the messenger adapter recomputes them on the
// host) and, when it was to store the results in h_out itself, that it did
// (PECH_FLAT_PUB; missing: the results come from the device's out[] by a
// copy).  Either way no CRC the kernel did not publish for this launch
// reaches a callback.  Both are counted (crc32c_async_get_stats).
static int slot_verify(crc32c_async *a, Slot *s)
{
	if (!s->flat_tag || !s->h_stat)
		return 0;
	const uint64_t v = __atomic_load_n(s->h_stat, __ATOMIC_ACQUIRE);
	if (v == PECH_FLAT_ERR(s->flat_tag)) {
		a->faults++;
		pech_internal_set_err("crc32c_async: a flat launch voided its results (its wait for out[] timed out)");
		return -EIO;
	}
	if (!s->published || v == PECH_FLAT_PUB(s->flat_tag))
		return 0;
	a->pub_missing++;
	int cur = -1;
	if (hipGetDevice(&cur) != hipSuccess)
		cur = -1;
	hipError_t e = hipSetDevice(a->dev);
	if (e == hipSuccess)
		e = hipMemcpyAsync(s->h_out, s->d_out, s->pieces.size() * 4u, hipMemcpyDeviceToHost, s->stream);
	if (e == hipSuccess)
		e = hipStreamSynchronize(s->stream);
	if (cur >= 0)
		(void)hipSetDevice(cur);
	if (e != hipSuccess) {
		pech_internal_set_err("crc32c_async: results copy after a missing publication failed: %s",
				      hipGetErrorString(e));
		return -EIO;
	}
	return 0;
}

// Harvest finished slots (blocking on the oldest when `wait`), in order.
static int reap(crc32c_async *a, bool wait_oldest, DeviceGuard *dg = nullptr)
{
	while (!a->inflight.empty()) {
		Slot *s = a->inflight.front();
		if (s->queued) { // CRC32C_ASYNC_DMA: the slots before it are harvested, so it launches now
			if (a->err) { // (a sticky error: it never launches)
				a->inflight.pop_front();
				harvest(a, s, a->err);
				if (wait_oldest)
					return a->err;
				continue;
			}
			if (dg && !dg->ensure())
				return 0;
			const int rc = issue_slot(a, s);
			if (rc) {
				if (wait_oldest)
					return rc;
				continue;
			}
			if (!wait_oldest)
				return 0; // just launched
		}
		hipError_t q = hipSuccess;
		if (wait_oldest) {
			// sleep until the host function marks the slot; a failed stream
			// never runs it, so the stream is asked every 2 ms
			s->waiting.store(1, std::memory_order_seq_cst);
			while (!s->finished.load(std::memory_order_seq_cst)) {
				flag_sleep(&s->finished, 2000000);
				if (s->finished.load(std::memory_order_seq_cst))
					break;
				q = hipStreamQuery(s->stream);
				if (q == hipSuccess && s->inject_fail)
					q = hipErrorLaunchFailure; // test build: as a failed stream reports itself
				if (q != hipSuccess && q != hipErrorNotReady)
					break; // failed: its host function will not run
				(void)hipGetLastError();
				q = hipSuccess; // (done but not yet marked: the flag comes next)
			}
			s->waiting.store(0, std::memory_order_relaxed);
		} else if (!s->finished.load(std::memory_order_acquire)) {
			// a failed stream never runs its host function: ask the stream,
			// once the batch has had kQueryAfterNs to finish (complete() is
			// called from the fd and from a timer; a query costs the caller's
			// thread microseconds, and the fd normally fires first)
			if (mono_ns() - s->t_launch < kQueryAfterNs || (dg && !dg->ensure()))
				return 0;
			q = hipStreamQuery(s->stream);
			if (q == hipSuccess && s->inject_fail)
				q = hipErrorLaunchFailure; // test build: as a failed stream reports itself
			if (q == hipSuccess || q == hipErrorNotReady) {
				(void)hipGetLastError();
				return 0;
			}
		}
		int err = 0;
		if (q != hipSuccess) {
			pech_internal_set_err("crc32c_async: batch failed: %s", hipGetErrorString(q));
			err = -EIO;
			a->err = err;
		} else {
			err = slot_verify(a, s); // (not sticky: the next batch is unaffected)
		}
		a->inflight.pop_front();
		harvest(a, s, err);
		if (wait_oldest) {
			// CRC32C_ASYNC_DMA: the next slot in line waited for this one;
			// it launches now, so the copy engine and the GPU work while the
			// caller fills the slot it waited for (it used to wait
			// for the next complete() or blocking get_slot)
			if (!err && !a->err && !a->inflight.empty() && a->inflight.front()->queued && (!dg || dg->ensure()))
				(void)issue_slot(a, a->inflight.front()); // (a failure is sticky in a->err)
			return err;
		}
	}
	return 0;
}

static int get_slot(crc32c_async *a, Slot **out)
{
	if (a->cur) {
		*out = a->cur;
		return 0;
	}
	for (Slot *s : a->slots)
		if (!s->inflight) {
			a->cur = *out = s;
			return 0;
		}
	if (a->slots.size() < a->max_slots) {
		Slot *s = slot_new(a->efd);
		if (!s)
			return -ENOMEM;
		a->slots.push_back(s);
		a->cur = *out = s;
		return 0;
	}
	// every slot in flight: wait for the oldest (callbacks still run only
	// in crc32c_async_complete)
	int rc;
	{
		ProfScope ps(a, 2);
		rc = reap(a, true);
	}
	if (rc)
		return rc;
	return get_slot(a, out);
}

// The slot being filled cannot be launched: its payloads fail (err), the
// context's error becomes sticky, and the eventfd wakes the loop so that
// crc32c_async_complete() delivers them.
static int fail_cur_slot(crc32c_async *a, int err)
{
	if (Slot *s = a->cur) {
		harvest(a, s, err);
		a->cur = nullptr;
	}
	a->err = err;
	const uint64_t one = 1;
	ssize_t r = write(a->efd, &one, sizeof(one));
	(void)r;
	return err;
}

// A slot that cannot be launched: the one being filled (fail_cur_slot), or
// a queued one, which is the oldest in flight when reap() launches it.
static int fail_slot(crc32c_async *a, Slot *s, int err)
{
	if (s == a->cur)
		return fail_cur_slot(a, err);
	if (!a->inflight.empty() && a->inflight.front() == s)
		a->inflight.pop_front();
	harvest(a, s, err);
	a->err = err;
	const uint64_t one = 1;
	ssize_t r = write(a->efd, &one, sizeof(one));
	(void)r;
	return err;
}

// Copies, descriptors, kernels, results and the host function of slot s:
// the slot being filled, or a queued one (CRC32C_ASYNC_DMA, from reap()).
static int issue_slot(crc32c_async *a, Slot *s)
{
	const unsigned m = (unsigned)s->pieces.size();
	a->launches++;
	ProfScope ps_copies(a, 0);
	if (!s->dma.empty()) {
		hipError_t e = hipErrorInvalidValue;
		if (!pech_fault(PECH_FAULT_ASYNC_DMA)) {
			e = hipErrorNotSupported;
			if (batch_copy_fn bc = batch_copy()) {
				std::vector<void *> dsts, srcs;
				std::vector<size_t> sizes;
				for (const DmaCopy &c : s->dma) {
					dsts.push_back(c.dst);
					srcs.push_back(c.src);
					sizes.push_back(c.bytes);
				}
				size_t fail_idx = SIZE_MAX;
				e = bc(dsts.data(), srcs.data(), sizes.data(), dsts.size(), nullptr, nullptr, 0, &fail_idx,
				       s->stream);
				// On a failure the per-copy calls issue EVERY copy again, from
				// copy 0: fail_idx only says where the batched call
				// stopped, not that the copies before it were queued, and a copy
				// never issued would leave stale staging bytes under a "good"
				// CRC; issuing a copy twice on one stream is harmless (the same
				// bytes land twice).
				if (e != hipSuccess && e != hipErrorNotSupported && e != hipErrorInvalidValue) {
					static std::once_flag warned;
					const hipError_t e0 = e;
					std::call_once(warned, [&] {
						fprintf(stderr, "pech_crc32c: hipMemcpyBatchAsync failed at copy %zu: %s; "
								"issuing every copy again, one call each\n",
							fail_idx, hipGetErrorString(e0));
					});
				}
			}
			if (e != hipSuccess) { // no batched call in this runtime (or it refused): one call each
				(void)hipGetLastError();
				e = hipSuccess;
				for (size_t k = 0; k < s->dma.size(); ++k) {
					const DmaCopy &c = s->dma[k];
					if ((e = hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyHostToDevice, s->stream)) !=
					    hipSuccess)
						break;
				}
			}
		}
		if (e != hipSuccess) {
			pech_internal_set_err("crc32c_async: payload DMA failed: %s", hipGetErrorString(e));
			return fail_slot(a, s, -EIO);
		}
	}
	for (auto &r : s->packed)
		TRY_HIP(hipMemcpyAsync(s->d_stage + r.first, s->h_stage + r.first, r.second - r.first,
				       hipMemcpyHostToDevice, s->stream),
			fail_slot(a, s, -EIO));
	const pech_desc *descs = s->desc_view;
	if (!descs) {
		TRY_HIP(hipMemcpyAsync(s->d_desc, s->h_desc, m * sizeof(pech_desc), hipMemcpyHostToDevice, s->stream),
			fail_slot(a, s, -EIO));
		descs = s->d_desc;
	}
	ps_copies.stop();
	ProfScope ps_launch(a, 1);
	s->finished.store(0, std::memory_order_relaxed);
	if (pech_fault(PECH_FAULT_ASYNC_LAUNCH)) {
		pech_internal_set_err("crc32c_async: injected launch failure (test)");
		return fail_slot(a, s, -EIO);
	}
	// results: stored into h_out by the flat and direct kernels themselves
	// (rc 1: no copy after them -- a blit kernel and its dispatch, ~4-5 us of
	// a lone payload's latency, profiles/r05/lat_prof.txt), else copied
	int rc = pech_internal_launch(descs, s->d_out, m, s->d_ws, pech_ws_bytes(kSlotDescs), s->stream,
				      s->maxlen < kDirectMax && !a->planned_only, s->out_view, s->stat_view, &s->flat_tag,
				      s->used == 0 && s->zc_bytes > 0 /* every piece read in place from pinned pages */);
	if (rc < 0)
		return fail_slot(a, s, rc);
	s->published = rc == 1 && s->flat_tag != 0;
	if (rc == 0)
		TRY_HIP(hipMemcpyAsync(s->h_out, s->d_out, m * 4u, hipMemcpyDeviceToHost, s->stream),
			fail_slot(a, s, -EIO));
	else
		a->host_out++;
	// test build: a batch whose stream fails after the launch -- HIP then
	// skips its host function, so the eventfd stays quiet
	s->inject_fail = pech_fault(PECH_FAULT_ASYNC_STREAM);
	bool poll = a->notify == 1 || a->notify == 2;
	if (a->notify == 3) { // a lone, small batch: polled
		unsigned others = 0;
		for (const Slot *o : a->inflight)
			others += o != s && !o->queued;
		poll = others == 0 && s->used + s->zc_bytes <= kPollMax;
	}
	if (!poll) {
		if (!s->inject_fail)
			TRY_HIP(hipLaunchHostFunc(s->stream, host_notify, s), fail_slot(a, s, -EIO));
	} else {
		s->est_ns = 8000u + (uint64_t)((s->used + s->zc_bytes) / 40u); // (40 bytes/ns: the host link)
		if (!s->ev_done)
			TRY_HIP(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming |
									(a->notify == 1 ? hipEventBlockingSync : 0u)),
				fail_slot(a, s, -EIO));
		TRY_HIP(hipEventRecord(s->ev_done, s->stream), fail_slot(a, s, -EIO));
		{
			std::lock_guard<std::mutex> lk(a->nmu);
			a->nq.push_back(s);
		}
		a->polled++;
		a->ncv.notify_one();
	}
	s->t_launch = mono_ns();
	if (s->queued) {
		s->queued = false; // (already in a->inflight, in order)
	} else {
		s->inflight = true;
		a->inflight.push_back(s);
		a->cur = nullptr;
	}
	return 0;
}

static int launch_slot(crc32c_async *a)
{
	Slot *s = a->cur;
	if (!s || s->pieces.empty())
		return 0;
	if ((a->flags & CRC32C_ASYNC_DMA) && !a->inflight.empty()) {
		// One slot's copies in flight at a time: with more, the runtime's
		// copy calls spin on the caller's thread (36-70 us of its CPU per
		// 4 MiB payload at 2-4 slots, 5 us at one; and 28-37 against 43
		// GiB/s; profiles/r04/async_dma_slots.txt).  The filled slot waits,
		// without a HIP call, until reap() has harvested the ones before it
		// -- complete() runs on the eventfd their host functions write.
		s->queued = true;
		s->inflight = true;
		a->inflight.push_back(s);
		a->cur = nullptr;
		return 0;
	}
	return issue_slot(a, s);
}

// The notifier thread (notify modes 1, 2): waits for each launched slot's
// event in launch order and does what the host function would (host_notify).
// A failed batch is left to reap()'s stream query, as with the host function,
// which HIP skips on a failed stream.
static void notifier_main(crc32c_async *a)
{
	(void)hipSetDevice(a->dev);
	(void)prctl(PR_SET_TIMERSLACK, 1000ul, 0ul, 0ul, 0ul); // 1 us: the predictive sleep wakes on time
	for (;;) {
		Slot *s;
		{
			std::unique_lock<std::mutex> lk(a->nmu);
			a->ncv.wait(lk, [a] { return a->nstop || !a->nq.empty(); });
			if (a->nq.empty())
				return; // (stop, nothing left)
			s = a->nq.front();
			a->nq.pop_front();
		}
		hipError_t e;
		if (a->notify == 1) {
			e = hipEventSynchronize(s->ev_done);
		} else {
			// sleep through ~70 % of the expected time (this thread's timer
			// slack is 1 us), then poll; a batch far beyond its estimate (a
			// slow link, a busy GPU) is polled every 20 us
			const uint64_t t0 = mono_ns();
			if (s->est_ns > 30000u) {
				const uint64_t ns = s->est_ns * 7u / 10u - 10000u;
				struct timespec ts = {(time_t)(ns / 1000000000u), (long)(ns % 1000000000u)};
				while (nanosleep(&ts, &ts) && errno == EINTR) {
				}
			}
			while ((e = hipEventQuery(s->ev_done)) == hipErrorNotReady) {
				// destroy: it has drained every slot before it asks
				// the thread to stop, so a batch still polled then never
				// completes (a failed stream's reap() already failed its
				// payloads): give up on it rather than block the join
				if (a->nstop.load(std::memory_order_relaxed))
					break;
				if (mono_ns() - t0 > 2 * s->est_ns + 100000u) {
					struct timespec ts = {0, 20000};
					nanosleep(&ts, nullptr);
				} else {
					__builtin_ia32_pause();
				}
			}
		}
		if (e == hipSuccess && !s->inject_fail)
			host_notify(s);
		else
			(void)hipGetLastError();
	}
}

static struct crc32c_async *async_create(unsigned int flags)
{
	if ((flags & ~(CRC32C_ASYNC_ZEROCOPY | CRC32C_ASYNC_DMA)) ||
	    (flags & (CRC32C_ASYNC_ZEROCOPY | CRC32C_ASYNC_DMA)) == (CRC32C_ASYNC_ZEROCOPY | CRC32C_ASYNC_DMA)) {
		pech_internal_set_err("crc32c_async_create: invalid flags %#x", flags);
		return nullptr;
	}
	if (crc32c_device_init())
		return nullptr;
	crc32c_async *a = new crc32c_async();
	a->flags = flags;
	const char *pl = getenv("PECH_ASYNC_PLANNED");
	a->planned_only = pl && pl[0] == '1';
	if (const char *zm = getenv("PECH_ASYNC_ZC_MAX"))
		a->zc_max = (size_t)strtoull(zm, nullptr, 0);
	if (const char *ms = getenv("PECH_ASYNC_SLOTS")) {
		const unsigned v = (unsigned)strtoul(ms, nullptr, 0);
		a->max_slots = v >= 1u && v <= kMaxSlots ? v : kMaxSlots;
	}
	if (hipGetDevice(&a->dev) != hipSuccess) {
		pech_internal_set_err("crc32c_async_create: %s", hipGetErrorString(hipGetLastError()));
		crc32c_async_destroy(a);
		return nullptr;
	}
	const char *pf = getenv("PECH_ASYNC_PROF");
	a->prof = pf && pf[0] == '1';
	if (const char *nm = getenv("PECH_ASYNC_NOTIFY"))
		a->notify = nm[0] >= '0' && nm[0] <= '3' ? nm[0] - '0' : 3;
	a->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
	if (a->efd < 0) {
		pech_internal_set_err("crc32c_async_create: eventfd: %s", strerror(errno));
		crc32c_async_destroy(a);
		return nullptr;
	}
	if (a->notify) {
		//  no exception may cross the C-ABI: without a thread
		// every batch is notified by a host function (mode 0)
		try {
			a->notifier = std::thread(notifier_main, a);
		} catch (...) {
			a->notify = 0;
		}
	}
	a->ready = true;
	return a;
}

extern "C" struct crc32c_async *crc32c_async_create(unsigned int flags)
{
	struct crc32c_async *a = nullptr;
	on_lib_stack([&] {
		a = async_create(flags);
		return 0;
	});
	return a;
}

extern "C" struct crc32c_async *crc32c_async_create_on(int device, unsigned int flags)
{
	struct crc32c_async *a = nullptr;
	on_lib_stack([&] {
		int ndev = 0;
		if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
			(void)hipGetLastError();
			pech_internal_set_err("crc32c_async_create_on: no device %d", device);
			return 0;
		}
		DeviceGuard dg(device);
		if (!dg.ok) {
			pech_internal_set_err("crc32c_async_create_on: cannot select device %d", device);
			return 0;
		}
		a = async_create(flags);
		return 0;
	});
	return a;
}

extern "C" int crc32c_async_devices(int *devs, int max)
{
	if (!devs || max <= 0) {
		pech_internal_set_err("crc32c_async_devices: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] { return pech_internal_device_list(devs, max < 64 ? max : 64, 16); });
}

extern "C" int crc32c_async_get_stats(const struct crc32c_async *a, struct crc32c_async_stats *st)
{
	if (!a || !st) {
		pech_internal_set_err("crc32c_async_get_stats: invalid arguments");
		return -EINVAL;
	}
	st->device = a->dev;
	st->submitted = a->submitted;
	st->launches = a->launches;
	st->host_out = a->host_out;
	st->polled = a->polled;
	st->faults = a->faults;
	st->pub_missing = a->pub_missing;
	st->inflight = st->queued = 0;
	for (const Slot *s : a->inflight)
		(s->queued ? st->queued : st->inflight)++;
	return 0;
}

extern "C" int crc32c_async_fd(const struct crc32c_async *a)
{
	return a ? a->efd : -EINVAL;
}

static int async_submit(struct crc32c_async *a, const void *buf, unsigned int len, uint32_t seed,
			crc32c_done_fn done, void *arg)
{
	// one registry lookup: pinned pages are read in place (zero-copy, below
	// kZeroCopyMax) or, with CRC32C_ASYNC_DMA, DMA'd
	const uint64_t dv = len ? pinned_dev_addr(buf, len) : 0;
	const uint64_t zc = !(a->flags & CRC32C_ASYNC_DMA) && len < a->zc_max ? dv : 0;
	const bool dma = !zc && dv != 0 && len >= kDmaMin;
	// the common case needs no HIP call: one descriptor (and, with
	// CRC32C_ASYNC_DMA, one recorded copy) into the open slot, which it does
	// not fill
	const Slot *c = a->cur;
	const bool quiet = c && c->pieces.size() + 1u < kSlotDescs && (zc ? c->zc_bytes + len < kSlotBytes : c->used + len + 512u < kSlotBytes);
	DeviceGuard dg(a->dev, !quiet);
	if (!quiet && !dg.ok) {
		pech_internal_set_err("crc32c_async_submit: cannot select device %d", a->dev);
		return -ENODEV;
	}
	const uint64_t id = a->base + a->items.size();
	a->items.push_back(Item{done, arg, seed, 0u, 0u, false, 0, false});
	const uint8_t *p = (const uint8_t *)buf;
	size_t left = len;
	uint32_t placed = 0;
	// A failure part-way: the pieces already placed complete (with an error
	// if their slot failed) and the item is retired without a callback.
	auto fail = [&](int rc) {
		Item &it = a->items[id - a->base];
		it.placed = true;
		it.total = placed;
		it.cancelled = true;
		return rc;
	};
	do {
		Slot *s = nullptr;
		int rc = get_slot(a, &s);
		if (rc)
			return fail(rc);
		if (s->pieces.size() == kSlotDescs || (!zc && left && s->used >= kSlotBytes)) {
			if ((rc = launch_slot(a)))
				return fail(rc);
			continue;
		}
		pech_desc &d = s->h_desc[s->pieces.size()];
		size_t piece;
		if (zc) {
			piece = left; // read in place: no staging space
			d.addr = zc + (len - left);
			s->zc_bytes += piece;
		} else {
			piece = left < kSlotBytes - s->used ? left : kSlotBytes - s->used;
			d.addr = (uint64_t)(uintptr_t)(s->d_stage + s->used);
			if (piece && dma) {
				// issued with the slot's other copies at launch: no HIP
				// call here (one each cost the caller 5-115 us)
				s->dma.push_back(DmaCopy{s->d_stage + s->used, const_cast<uint8_t *>(p), piece});
			} else if (piece) {
				memcpy(s->h_stage + s->used, p, piece);
				if (!s->packed.empty() && s->packed.back().second == s->used)
					s->packed.back().second = s->used + piece;
				else
					s->packed.push_back({s->used, s->used + piece});
			}
			s->used = (s->used + piece + 255u) & ~(size_t)255u;
		}
		d.len = (uint32_t)piece;
		d.seed = placed == 0 ? seed : 0u;
		s->pieces.push_back(Piece{id, (uint32_t)piece});
		s->maxlen = s->maxlen > piece ? s->maxlen : (uint32_t)piece;
		++placed;
		p += piece;
		left -= piece;
	} while (left);
	Item &it = a->items[id - a->base];
	it.placed = true;
	it.total = placed;
	a->submitted++;
	Slot *s = a->cur;
	if (s && (s->pieces.size() == kSlotDescs || s->used >= kSlotBytes || s->zc_bytes >= kSlotBytes)) {
		const int rc = launch_slot(a);
		// This payload filled the slot and its launch failed: its pieces are
		// harvested with the error, but the submission returns it, so the
		// item is retired without a callback (error return and callback are
		// exclusive; the caller still owns the bytes and recomputes).
		if (rc)
			a->items[id - a->base].cancelled = true;
		return rc;
	}
	return 0;
}

extern "C" int crc32c_async_submit(struct crc32c_async *a, const void *buf, unsigned int len, uint32_t seed,
				   crc32c_done_fn done, void *arg)
{
	if (!a || !done || (len && !buf)) {
		pech_internal_set_err("crc32c_async_submit: invalid arguments");
		return -EINVAL;
	}
	if (a->err)
		return a->err;
	ProfScope ps(a, 3);
	return on_lib_stack([&] { return async_submit(a, buf, len, seed, done, arg); });
}

// The messenger adapter's queue-depth signal (crc32c_msgr.c route_host): a
// payload is "lone" when nothing is outstanding on the context and no other
// was taken as lone since the last flush -- the patched messenger flushes at
// the end of every con_work pass, so a burst read in one pass sends its
// first payload to the host and the rest to the GPU, while queue depth 1
// (one message per pass) sends every one to the host.
extern "C" PECH_HIDDEN int pech_async_take_lone(struct crc32c_async *a)
{
	if (!a || !a->items.empty() || a->lone_taken)
		return 0;
	a->lone_taken = true;
	return 1;
}

extern "C" int crc32c_async_flush(struct crc32c_async *a)
{
	if (!a)
		return -EINVAL;
	a->lone_taken = false; // (a new pass: see pech_async_take_lone)
	if (a->err)
		return a->err;
	if (!a->cur || a->cur->pieces.empty())
		return 0; // nothing to launch: no device guard, no stack switch
	return on_lib_stack([&] {
		DeviceGuard dg(a->dev);
		return launch_slot(a);
	});
}

// items are finished when every placed piece has been harvested; runs on
// the caller's stack and device
static int run_callbacks(crc32c_async *a)
{
	int ran = 0;
	while (!a->items.empty()) {
		Item &it = a->items.front();
		if (!it.placed || it.harvested != it.total)
			break;
		const Item done = it;
		a->items.pop_front();
		a->base++;
		if (done.cancelled)
			continue;
		done.done(done.arg, done.err ? 0u : done.crc, done.err);
		++ran;
	}
	return ran;
}

extern "C" int crc32c_async_complete(struct crc32c_async *a)
{
	if (!a)
		return -EINVAL;
	ProfScope ps(a, 4);
	const int rc = on_lib_stack([&] {
		uint64_t cnt;
		while (read(a->efd, &cnt, sizeof(cnt)) > 0) {
		}
		DeviceGuard dg(a->dev, false); // reap() selects it before a stream query
		return reap(a, false, &dg);
	});
	const int ran = run_callbacks(a);
	return rc ? rc : ran;
}

extern "C" int crc32c_async_drain(struct crc32c_async *a)
{
	if (!a)
		return -EINVAL;
	const int rc = on_lib_stack([&] {
		DeviceGuard dg(a->dev);
		int r0 = a->err ? a->err : launch_slot(a);
		if (a->err && a->cur) // a sticky error: what was never launched fails now
			fail_cur_slot(a, a->err);
		while (!a->inflight.empty()) {
			int r = reap(a, true);
			if (r && !r0)
				r0 = r;
		}
		if (!r0)
			r0 = a->err; // (e.g. a queued slot that reap() launched and that failed)
		uint64_t cnt;
		while (read(a->efd, &cnt, sizeof(cnt)) > 0) {
		}
		return r0;
	});
	run_callbacks(a);
	return rc;
}

extern "C" unsigned int crc32c_async_pending(const struct crc32c_async *a)
{
	return a ? (unsigned int)a->items.size() : 0u;
}

extern "C" void crc32c_async_destroy(struct crc32c_async *a)
{
	if (!a)
		return;
	if (a->ready)
		(void)crc32c_async_drain(a); // callbacks on the caller's stack
	if (a->notifier.joinable()) {
		{
			std::lock_guard<std::mutex> lk(a->nmu);
			a->nstop = true;
		}
		a->ncv.notify_one();
		a->notifier.join();
	}
	on_lib_stack([&] {
		DeviceGuard dg(a->dev >= 0 ? a->dev : 0);
		for (Slot *s : a->slots)
			slot_free(s); // synchronises the slot's stream first
		return 0;
	});
	if (a->prof)
		fprintf(stderr,
			"{\"async_prof\": {\"launches\": %llu, \"thread_cpu_us\": {\"copies\": %.1f, \"launch\": %.1f, "
			"\"slot_wait\": %.1f, \"submit\": %.1f, \"complete\": %.1f}}}\n",
			(unsigned long long)a->launches, a->prof_ns[0] / 1e3, a->prof_ns[1] / 1e3, a->prof_ns[2] / 1e3,
			a->prof_ns[3] / 1e3, a->prof_ns[4] / 1e3);
	if (a->efd >= 0)
		close(a->efd);
	delete a;
}
