// crc32c_api.cpp -- C-ABI of libpech_crc32c.so (include/crc32c.h,
// include/pech_crc32c.h): per-device context, constant tables, launch
// sequencing, host-memory staging pipeline.
//
// Every batch, device and async entry point computes on the gfx950 kernels
// (crc32c_kernels.hip) and reports a HIP failure as -EIO; this file moves
// bytes and descriptors.  The one exception is the drop-in crc32c(): like
// the reference (include/crc32c.h:88-96) it cannot fail, so calls up to
// crc32c_set_cpu_max() bytes (the messenger's headers, front sections and
// <=4 KiB pieces) run on the host routine of
// crc32c_cpu.c, and a failed GPU call is recomputed there (counted in
// crc32c_get_stats(), reported once on stderr).
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/pech_crc32c.h"
#include "api_internal.h"
#include "gf2.h"
#include "layout.h"

static_assert(sizeof(struct crc32c_desc) == sizeof(struct pech_desc), "descriptor ABI");
static_assert(sizeof(struct crc32c_desc) == 16, "descriptor ABI");

extern "C" hipError_t pech_launch_plan(const pech_desc *, uint32_t, const pech_ws *, const uint32_t *, uint32_t *,
				       const uint64_t *, hipStream_t);
extern "C" hipError_t pech_launch_main(uint32_t, const pech_ws *, const uint32_t *, uint32_t *, uint32_t, uint32_t, int,
				       hipStream_t, hipEvent_t, hipEvent_t);

extern "C" const char *pech_kernel_tag(void);
extern "C" hipError_t pech_launch_direct(const pech_desc *, uint32_t, const uint32_t *, uint32_t *, uint32_t,
					 hipStream_t, hipEvent_t, hipEvent_t, const uint64_t *);
extern "C" hipError_t pech_launch_small(const void *, uint32_t, uint32_t, const uint32_t *, uint32_t *, uint32_t,
					hipStream_t);
extern "C" hipError_t pech_launch_flat(const pech_desc *, uint32_t, const uint32_t *, uint32_t *, uint32_t, uint32_t,
				       uint64_t *, uint64_t, hipStream_t, hipEvent_t, hipEvent_t, uint32_t *, uint64_t *,
				       uint32_t);
extern "C" int pech_read_flat_faults(uint64_t *);

// ---------------------------------------------------------------------------
static thread_local char g_err[512];

static void set_err(const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof(g_err), fmt, ap);
	va_end(ap);
}

#define HIP_TRY(expr)                                                                          \
	do {                                                                                   \
		hipError_t e_ = (expr);                                                        \
		if (e_ != hipSuccess) {                                                        \
			set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
				__LINE__);                                                     \
			return -EIO;                                                           \
		}                                                                              \
	} while (0)

// ---------------------------------------------------------------------------
// constant tables (host side, built once)
static void build_consts(uint32_t *c)
{
	// byte tables of A_n (advance n zero bytes): T_k[e] = A_n(e << 8k)
	const uint64_t shifts[5] = {128, 4, 16, 32, 64}; // TAB128, TAB4, TAB16, TAB32, TAB64
	for (int t = 0; t < 5; ++t) {
		const uint32_t xk = gf2_x8n(shifts[t]);
		for (uint32_t k = 0; k < 4; ++k)
			for (uint32_t e = 0; e < 256; ++e)
				c[t * 1024u + k * 256u + e] = gf2_mulmod(xk, e << (8 * k));
	}
	// POWB[i][j] = x^(8 * j * 64^i)
	for (uint32_t i = 0; i < 6; ++i) {
		const uint32_t base = gf2_x8n((uint64_t)1 << (6 * i));
		uint32_t acc = CRC32C_ONE;
		for (uint32_t j = 0; j < 64; ++j) {
			c[PECH_C_POWB + 64 * i + j] = acc;
			acc = gf2_mulmod(acc, base);
		}
	}
	// A_1: the reference byte table (include/crc32c.h:16-81), regenerated
	for (uint32_t e = 0; e < 256; ++e)
		c[PECH_C_TAB1 + e] = gf2_mulmod(CRC32C_X8, e);
	// A_16384: the fused copy's Horner step over rows 128 apart (interleaved mode)
	{
		const uint32_t xk = gf2_x8n((uint64_t)PECH_IL_GROUPS * PECH_ROW_BYTES);
		for (uint32_t k = 0; k < 4; ++k)
			for (uint32_t e = 0; e < 256; ++e)
				c[PECH_C_TAB16K + k * 256u + e] = gf2_mulmod(xk, e << (8 * k));
	}
	// ROWPOW[k] = x^(8 * 128 k) = A_128^k(1), by the A_128 byte tables
	c[PECH_C_ROWPOW] = CRC32C_ONE;
	for (uint32_t k = 1; k < PECH_ROWPOW_N; ++k) {
		const uint32_t v = c[PECH_C_ROWPOW + k - 1];
		c[PECH_C_ROWPOW + k] = c[PECH_C_TAB128 + (v & 0xFFu)] ^ c[PECH_C_TAB128 + 256u + ((v >> 8) & 0xFFu)] ^
				       c[PECH_C_TAB128 + 512u + ((v >> 16) & 0xFFu)] ^ c[PECH_C_TAB128 + 768u + (v >> 24)];
	}
	// XINV[k] = x^(-8k): undoes k trailing zero bytes (a core's last line)
	const uint32_t xinv8 = gf2_xinv8n(1);
	uint32_t acc = CRC32C_ONE;
	for (uint32_t k = 0; k < 128; ++k) {
		c[PECH_C_XINV + k] = acc;
		acc = gf2_mulmod(acc, xinv8);
	}
}

// ---------------------------------------------------------------------------
struct TimedLaunch {
	hipEvent_t a, b;
};

struct DevCtx {
	int dev = -1;
	int ncu = 0;
	uint32_t *d_consts = nullptr;
	// internal workspace of crc32c_dev_[copy_]batch_async, which run on the
	// CALLER's streams: the last launch that used it is recorded in ws_ev, and
	// a launch on another stream waits for it (never two launches at once)
	void *d_ws = nullptr;
	size_t ws_bytes = 0;
	hipEvent_t ws_ev = nullptr;
	hipStream_t ws_stream = nullptr;
	bool ws_used = false;
	// workspace of the synchronous host paths, used on s_comp only
	void *d_ws_host = nullptr;
	size_t ws_host_bytes = 0;
	// synchronous host paths
	hipStream_t s_comp = nullptr, s_copy[2] = {nullptr, nullptr}; // one copy stream per staging slot
	uint8_t *h_stage[2] = {nullptr, nullptr};
	uint8_t *d_stage[2] = {nullptr, nullptr};
	size_t stage_bytes = 0;
	pech_desc *h_desc[2] = {nullptr, nullptr};
	pech_desc *d_desc[2] = {nullptr, nullptr};
	uint32_t *h_out[2] = {nullptr, nullptr};
	uint32_t *d_out[2] = {nullptr, nullptr};
	uint32_t desc_cap = 0;
	hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
	// drop-in small path: device views of h_stage[0] and h_out[0] (zero-copy)
	void *small_src = nullptr;
	uint32_t *h_small = nullptr, *small_out = nullptr; // result + ticket, coherent pinned memory
	uint32_t small_ticket = 0;
	// flat launches' status words (layout.h PECH_FLAT_ERR), coherent pinned
	// memory: [0] the synchronous host paths' launches (checked after each
	// wait: flat_check), [1] the device entry points' (the caller reads
	// crc32c_get_stats().gpu_faults)
	uint64_t *h_stat = nullptr, *d_stat = nullptr;
	uint64_t stat_seen = 0; // h_stat[0] at the last flat_check
	// timing
	std::vector<TimedLaunch> pending;
	std::vector<TimedLaunch> free_events;
};

static std::mutex g_mu;
static DevCtx g_ctx[64];
static bool g_timing = false;
static std::vector<float> g_samples; // per-launch main-kernel ms of the last timing_read
static uint32_t g_host_consts[PECH_C_WORDS];
static bool g_host_consts_ready = false;

static const uint32_t *host_consts()
{
	if (!g_host_consts_ready) {
		build_consts(g_host_consts);
		g_host_consts_ready = true;
	}
	return g_host_consts;
}

static int ctx_get(DevCtx **out)
{
	int dev = 0;
	hipError_t e = hipGetDevice(&dev);
	if (e != hipSuccess) {
		set_err("no usable GPU: hipGetDevice: %s", hipGetErrorString(e));
		return -ENODEV;
	}
	if (dev < 0 || dev >= 64) {
		set_err("device index %d out of range", dev);
		return -ENODEV;
	}
	DevCtx *c = &g_ctx[dev];
	if (c->dev < 0) {
		hipDeviceProp_t prop;
		HIP_TRY(hipGetDeviceProperties(&prop, dev));
		c->ncu = prop.multiProcessorCount;
		HIP_TRY(hipMalloc(&c->d_consts, PECH_C_WORDS * sizeof(uint32_t)));
		HIP_TRY(hipMemcpy(c->d_consts, host_consts(), PECH_C_WORDS * sizeof(uint32_t), hipMemcpyHostToDevice));
		HIP_TRY(hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking));
		{ // fine-grained: the small kernel's system-scope stores are visible while it runs
			void *so = nullptr;
			HIP_TRY(hipHostMalloc((void **)&c->h_small, 256, hipHostMallocCoherent | hipHostMallocMapped));
			memset(c->h_small, 0, 256); // ticket 0 is never issued
			HIP_TRY(hipHostGetDevicePointer(&so, c->h_small, 0));
			c->small_out = (uint32_t *)so;
			HIP_TRY(hipHostMalloc((void **)&c->h_stat, 64, hipHostMallocCoherent | hipHostMallocMapped));
			memset(c->h_stat, 0, 64);
			HIP_TRY(hipHostGetDevicePointer(&so, c->h_stat, 0));
			c->d_stat = (uint64_t *)so;
		}
		for (int i = 0; i < 2; ++i) // two slots' copies may run on two DMA engines at once
			HIP_TRY(hipStreamCreateWithFlags(&c->s_copy[i], hipStreamNonBlocking));
		for (int i = 0; i < 2; ++i) {
			HIP_TRY(hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming));
			HIP_TRY(hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming));
		}
		HIP_TRY(hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming));
		c->dev = dev;
	}
	*out = c;
	return 0;
}

// workspace layout: layout.h (pech_ws_carve)
static size_t ws_bytes_for(unsigned int n)
{
	return pech_ws_bytes(n);
}

// the device-batch workspace (crc32c_dev_[copy_]batch_async): regrown only
// after the last launch that used it has finished
static int ws_reserve(DevCtx *c, unsigned int n)
{
	const size_t need = ws_bytes_for(n < PECH_MAX_BATCH ? n : PECH_MAX_BATCH);
	if (need <= c->ws_bytes)
		return 0;
	if (c->d_ws) {
		if (c->ws_used)
			HIP_TRY(hipEventSynchronize(c->ws_ev));
		HIP_TRY(hipFree(c->d_ws));
	}
	c->d_ws = nullptr;
	c->ws_bytes = 0;
	c->ws_used = false;
	HIP_TRY(hipMalloc(&c->d_ws, need));
	c->ws_bytes = need;
	return 0;
}

// the host paths' workspace, used on s_comp only
static int ws_host_reserve(DevCtx *c, unsigned int n)
{
	const size_t need = ws_bytes_for(n < PECH_MAX_BATCH ? n : PECH_MAX_BATCH);
	if (need <= c->ws_host_bytes)
		return 0;
	if (c->d_ws_host) {
		HIP_TRY(hipStreamSynchronize(c->s_comp));
		HIP_TRY(hipFree(c->d_ws_host));
	}
	c->d_ws_host = nullptr;
	c->ws_host_bytes = 0;
	HIP_TRY(hipMalloc(&c->d_ws_host, need));
	c->ws_host_bytes = need;
	return 0;
}

static bool capturing(hipStream_t s)
{
	hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
	if (hipStreamIsCapturing(s, &st) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	return st != hipStreamCaptureStatusNone;
}

// Batches of at most g_flat_max buffers run as ONE launch (pech_crc32c_flat
// up to 256 buffers, pech_crc32c_flatg above: no plan kernel) -- C3's 256 x 4 MiB, the async layer's slots of large
// payloads, a single large message.  Its workgroup 0 publishes the zeroed
// out[] through the first 8 bytes of the workspace and a tag that must differ
// from every earlier launch's on that workspace: a process-wide 64-bit
// counter from a per-process start, so a tag left in recycled memory by
// another run does not match either.  A graph replays its captured tag, so
// captured batches take plan + main.
// Default PECH_FLATG_MAX (4,096): since its prologue locates a uniform
// batch's shares by division and its first step plans from descriptors
// loaded at entry, pech_crc32c_flatg's one launch costs what plan + main did
// on one stream (c4-64k 4,628 / 4,625 against 4,630 / 4,624 GiB/s serial) and
// two streams gain 6-7 % (5,549-5,610 against 5,247-5,256; profiles/r06/flatg.txt).
static std::atomic<unsigned int> g_flat_max{PECH_FLATG_MAX};

// rows per wave below which a launch spreads its shares wave-major
// (crc32c_kernels.hip wave_share); PECH_RPW_MIN overrides it (A/B measurements)
static uint32_t rpw_min()
{
	static const uint32_t v = [] {
		const char *e = getenv("PECH_RPW_MIN");
		const unsigned long r = e ? strtoul(e, nullptr, 0) : 0ul;
		return r >= 8u && r <= 4096u ? (uint32_t)r : PECH_RPW_MIN;
	}();
	return v;
}
// PECH_FLAT_IL=0: host-resident flat launches keep static slices (A/B and
// tests; read at each such launch)
static bool flat_il()
{
	const char *e = getenv("PECH_FLAT_IL");
	return !(e && e[0] == '0');
}
static std::atomic<uint64_t> g_flat_tag{0};
static std::once_flag g_flat_tag_init;

static uint64_t flat_tag()
{
	std::call_once(g_flat_tag_init, [] {
		uint64_t t = 0;
		FILE *f = fopen("/dev/urandom", "rb");
		if (!f || fread(&t, sizeof(t), 1, f) != 1)
			t = (uint64_t)(uintptr_t)&t ^ ((uint64_t)clock() << 32) ^ 0x9E3779B97F4A7C15ull;
		if (f)
			fclose(f);
		g_flat_tag.store(t);
	});
	// below 2^62: the kernel keeps two states per tag in the 64-bit word
	// (tag << 1, tag << 1 | 1); 0 (a zeroed workspace's value) is skipped
	uint64_t t;
	while (((t = g_flat_tag.fetch_add(1) + 1) & ((1ull << 62) - 1u)) == 0)
		;
	return t & ((1ull << 62) - 1u);
}

// d_dsts != NULL: fused CRC + copy (d_dsts[i] receives descriptor i's bytes).
// hout != NULL (the async layer's slots): a flat launch also stores the
// results there, a device-visible pinned host array (*published = true).
// hstat: the device view of the status word a flat launch reports a fault
// (or its publication) in (layout.h PECH_FLAT_ERR / PECH_FLAT_PUB; NULL:
// the device entry points' word of the context); *flat_tag: the flat
// launch's tag (0: no flat launch).
// host_resident: every buffer is pinned host memory the kernel reads in place
// (an async zero-copy slot): flat launches of uniform large buffers then walk
// interleaved rows (PECH_FLAT_F_IL), the shape that reads the host link at the
// copy engines' rate.
static int launch_batch(DevCtx *c, const pech_desc *d_descs, uint32_t *d_out, unsigned int n, void *ws,
			size_t ws_bytes, hipStream_t stream, const uint64_t *d_dsts = nullptr, uint32_t *hout = nullptr,
			bool *published = nullptr, uint64_t *hstat = nullptr, uint64_t *flat_tag_out = nullptr,
			bool host_resident = false)
{
	if (flat_tag_out)
		*flat_tag_out = 0;
	if (n == 0)
		return 0;
	for (unsigned int off = 0; off < n; off += PECH_MAX_BATCH) {
		const unsigned int m = (n - off) < PECH_MAX_BATCH ? (n - off) : PECH_MAX_BATCH;
		if (ws_bytes < ws_bytes_for(m)) {
			set_err("workspace too small: %zu < %zu", ws_bytes, ws_bytes_for(m));
			return -EINVAL;
		}
		if ((uintptr_t)ws & 255u) {
			set_err("workspace must be 256-byte aligned");
			return -EINVAL;
		}
		const bool flat = !d_dsts && m <= g_flat_max.load(std::memory_order_relaxed) && !capturing(stream);
		const pech_ws w = pech_ws_carve(ws, m);
		if (!flat)
			HIP_TRY(pech_launch_plan(d_descs + off, m, &w, c->d_consts, d_out + off,
						 d_dsts ? d_dsts + off : nullptr, stream));
		TimedLaunch tl{};
		if (g_timing) {
			if (!c->free_events.empty()) {
				tl = c->free_events.back();
				c->free_events.pop_back();
			} else {
				HIP_TRY(hipEventCreate(&tl.a));
				HIP_TRY(hipEventCreate(&tl.b));
			}
		}
		if (flat)
		{
			const bool pub = hout && m == n; // (one launch: a flat batch is)
			// test library only: the kernel's fault bits (release: always 0)
			const uint32_t test = (pech_fault(PECH_FAULT_FLAT_TIMEOUT) ? PECH_FLAT_T_TIMEOUT : 0u) |
					      (pub && pech_fault(PECH_FAULT_FLAT_NOPUB) ? PECH_FLAT_T_NOPUB : 0u) |
					      (host_resident && flat_il() ? PECH_FLAT_F_IL : 0u);
			const uint64_t tag = flat_tag();
			HIP_TRY(pech_launch_flat(d_descs + off, m, c->d_consts, d_out + off, (uint32_t)c->ncu, rpw_min(),
						 (uint64_t *)ws, tag, stream, tl.a, tl.b, pub ? hout : nullptr,
						 hstat ? hstat : c->d_stat + 1, test));
			if (flat_tag_out)
				*flat_tag_out = tag;
			if (pub && published)
				*published = true;
		}
		else
			HIP_TRY(pech_launch_main(m, &w, c->d_consts, d_out + off, (uint32_t)c->ncu, rpw_min(),
						 d_dsts != nullptr, stream, tl.a, tl.b));
		if (g_timing)
			c->pending.push_back(tl);
	}
	return 0;
}

// After a synchronous host path has waited for its launches: a flat launch
// that reported a fault in the context's status word (layout.h
// PECH_FLAT_ERR; the word changes only then, and tags never repeat) voids
// the results of the call -- -EIO, and the drop-in recomputes on the host.
static int flat_check(DevCtx *c)
{
	const uint64_t v = __atomic_load_n(c->h_stat, __ATOMIC_ACQUIRE);
	if (v == c->stat_seen)
		return 0;
	c->stat_seen = v;
	(void)hipStreamSynchronize(c->s_comp); // nothing of the call still runs when it returns
	set_err("flat kernel: a wave's wait for out[]'s initialisation timed out; the batch's results are void");
	return -EIO;
}

// A device batch on the internal workspace, on the caller's stream: ordered
// after the previous user of the workspace when that was another stream
// (two streams must never share it concurrently).  Refused inside
// a graph capture: a replay would use the workspace outside this
// ordering, and a later reserve could free it under the graph -- captured
// batches take the _ws_ forms (own workspace) or crc32c_dev_batch_small_async
// (none).
static int launch_internal_ws(DevCtx *c, const pech_desc *d_descs, uint32_t *d_out, unsigned int n,
			      hipStream_t stream, const uint64_t *d_dsts)
{
	if (capturing(stream)) {
		set_err("the internal workspace cannot be captured in a graph: use the _ws_ forms "
			"(own workspace) or crc32c_dev_batch_small_async");
		return -EINVAL;
	}
	int rc = ws_reserve(c, n);
	if (rc)
		return rc;
	if (c->ws_used && c->ws_stream != stream)
		HIP_TRY(hipStreamWaitEvent(stream, c->ws_ev, 0));
	if ((rc = launch_batch(c, d_descs, d_out, n, c->d_ws, c->ws_bytes, stream, d_dsts)))
		return rc;
	HIP_TRY(hipEventRecord(c->ws_ev, stream));
	c->ws_stream = stream;
	c->ws_used = true;
	return 0;
}

// The direct kernel (no plan kernel, no workspace): small-buffer batches,
// in launches of at most PECH_MAX_BATCH descriptors (output slots are 20 bits)
static int launch_small(DevCtx *c, const pech_desc *d_descs, uint32_t *d_out, unsigned int n, hipStream_t stream,
			const uint64_t *d_dsts = nullptr)
{
	for (unsigned int off = 0; off < n; off += PECH_MAX_BATCH) {
		const unsigned int m = (n - off) < PECH_MAX_BATCH ? (n - off) : PECH_MAX_BATCH;
		TimedLaunch tl{};
		if (g_timing) {
			if (!c->free_events.empty()) {
				tl = c->free_events.back();
				c->free_events.pop_back();
			} else {
				HIP_TRY(hipEventCreate(&tl.a));
				HIP_TRY(hipEventCreate(&tl.b));
			}
		}
		HIP_TRY(pech_launch_direct(d_descs + off, m, c->d_consts, d_out + off, (uint32_t)c->ncu, stream, tl.a, tl.b,
					   d_dsts ? d_dsts + off : nullptr));
		if (g_timing)
			c->pending.push_back(tl);
	}
	return 0;
}

// ---------------------------------------------------------------------------
// internal entry points for crc32c_async.cpp (hidden: not part of the C-ABI)

PECH_HIDDEN int pech_internal_launch(const pech_desc *d_descs, uint32_t *d_out, unsigned int n, void *ws,
				     size_t ws_bytes, hipStream_t stream, bool small, uint32_t *hout, uint64_t *hstat,
				     uint64_t *flat_tag, bool host_resident)
{
	if (flat_tag)
		*flat_tag = 0;
	std::lock_guard<std::mutex> lk(g_mu);
	DevCtx *c = nullptr;
	int rc = ctx_get(&c);
	if (rc)
		return rc;
	if (small) // the direct kernel stores each result once: straight to the host array when there is one
		return hout && n <= PECH_MAX_BATCH ? (launch_small(c, d_descs, hout, n, stream) ?: 1)
						   : launch_small(c, d_descs, d_out, n, stream);
	bool pub = false;
	rc = launch_batch(c, d_descs, d_out, n, ws, ws_bytes, stream, nullptr, hout, &pub, hstat, flat_tag, host_resident);
	return rc ? rc : pub ? 1 : 0;
}

PECH_HIDDEN int pech_internal_device_list(int *devs, int max, int max_per_dev)
{
	int nd = 0;
	if (const char *e = getenv("PECH_DEVICES")) {
		for (const char *p = e; *p && nd < max;) {
			char *q = nullptr;
			const long v = strtol(p, &q, 10);
			if (q == p)
				break;
			devs[nd++] = (int)v;
			p = *q == ',' ? q + 1 : q;
		}
	} else {
		HIP_TRY(hipGetDeviceCount(&nd));
		nd = nd < max ? nd : max;
		for (int d = 0; d < nd; ++d)
			devs[d] = d;
	}
	int ndev_all = 0;
	HIP_TRY(hipGetDeviceCount(&ndev_all));
	int used[64] = {0};
	for (int k = 0; k < nd; ++k) {
		if (devs[k] < 0 || devs[k] >= ndev_all || devs[k] >= 64 || used[devs[k]] >= max_per_dev) {
			set_err("bad device list (PECH_DEVICES)");
			return -EINVAL;
		}
		used[devs[k]]++;
	}
	if (nd == 0) {
		set_err("no usable GPU");
		return -ENODEV;
	}
	return nd;
}

PECH_HIDDEN void pech_internal_set_err(const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof(g_err), fmt, ap);
	va_end(ap);
}

// ---------------------------------------------------------------------------
// host staging: two slots of `bytes` pinned host + device memory each
static int stage_reserve(DevCtx *c, size_t bytes, uint32_t ndesc)
{
	if (bytes > c->stage_bytes) {
		for (int i = 0; i < 2; ++i) {
			if (c->h_stage[i])
				HIP_TRY(hipHostFree(c->h_stage[i]));
			if (c->d_stage[i])
				HIP_TRY(hipFree(c->d_stage[i]));
			c->h_stage[i] = nullptr;
			c->d_stage[i] = nullptr;
		}
		c->stage_bytes = 0;
		for (int i = 0; i < 2; ++i) {
			HIP_TRY(hipHostMalloc(&c->h_stage[i], bytes, hipHostMallocDefault));
			HIP_TRY(hipMalloc(&c->d_stage[i], bytes));
		}
		c->stage_bytes = bytes;
		c->small_src = nullptr;
		HIP_TRY(hipHostGetDevicePointer(&c->small_src, c->h_stage[0], 0));
	}
	if (ndesc > c->desc_cap) {
		for (int i = 0; i < 2; ++i) {
			if (c->h_desc[i])
				HIP_TRY(hipHostFree(c->h_desc[i]));
			if (c->d_desc[i])
				HIP_TRY(hipFree(c->d_desc[i]));
			if (c->h_out[i])
				HIP_TRY(hipHostFree(c->h_out[i]));
			if (c->d_out[i])
				HIP_TRY(hipFree(c->d_out[i]));
			c->h_desc[i] = nullptr;
			c->d_desc[i] = nullptr;
			c->h_out[i] = nullptr;
			c->d_out[i] = nullptr;
		}
		c->desc_cap = 0;
		for (int i = 0; i < 2; ++i) {
			HIP_TRY(hipHostMalloc(&c->h_desc[i], (size_t)ndesc * sizeof(pech_desc), hipHostMallocDefault));
			HIP_TRY(hipMalloc(&c->d_desc[i], (size_t)ndesc * sizeof(pech_desc)));
			HIP_TRY(hipHostMalloc(&c->h_out[i], (size_t)ndesc * 4u, hipHostMallocDefault));
			HIP_TRY(hipMalloc(&c->d_out[i], (size_t)ndesc * 4u));
		}
		c->desc_cap = ndesc;
	}
	return 0;
}

static const size_t STAGE_BYTES = 64u << 20;      // per slot
static const uint32_t STAGE_DESCS = 1u << 16;     // per slot
static const size_t PINNED_DIRECT_MIN = 1u << 20; // pinned buffers >= this are DMA'd, smaller ones read in place

// One sub-batch of host buffers into slot `s`: gather bytes, enqueue copy,
// kernels and result copy.  Buffers must each fit the slot.
static int enqueue_host_slot(DevCtx *c, int s, const void *const *bufs, const unsigned int *lens,
			     const uint32_t *seeds, const uint32_t *chain_seed, unsigned int i0, unsigned int m,
			     unsigned int flags)
{
	size_t off = 0;
	size_t packed_lo = 0; // start of the pending host-packed run
	for (unsigned int k = 0; k < m; ++k) {
		const unsigned int i = i0 + k;
		const size_t len = lens[i];
		const bool direct = (flags & CRC32C_F_PINNED) && len >= PINNED_DIRECT_MIN;
		void *zc = nullptr; // small pinned buffer: the kernel reads it in place (no host memcpy)
		if ((flags & CRC32C_F_PINNED) && !direct && len &&
		    (hipHostGetDevicePointer(&zc, const_cast<void *>(bufs[i]), 0) != hipSuccess || !zc)) {
			(void)hipGetLastError();
			zc = nullptr;
		}
		if (zc) {
			c->h_desc[s][k].addr = (uint64_t)(uintptr_t)zc;
			c->h_desc[s][k].len = (uint32_t)len;
			c->h_desc[s][k].seed = chain_seed ? *chain_seed : (seeds ? seeds[i] : 0u);
			continue;
		}
		if (direct) {
			if (off > packed_lo)
				HIP_TRY(hipMemcpyAsync(c->d_stage[s] + packed_lo, c->h_stage[s] + packed_lo,
						       off - packed_lo, hipMemcpyHostToDevice, c->s_copy[s]));
			HIP_TRY(hipMemcpyAsync(c->d_stage[s] + off, bufs[i], len, hipMemcpyHostToDevice, c->s_copy[s]));
		} else if (len) {
			memcpy(c->h_stage[s] + off, bufs[i], len);
		}
		c->h_desc[s][k].addr = (uint64_t)(uintptr_t)(c->d_stage[s] + off);
		c->h_desc[s][k].len = (uint32_t)len;
		c->h_desc[s][k].seed = chain_seed ? *chain_seed : (seeds ? seeds[i] : 0u);
		off = (off + len + 255u) & ~(size_t)255u;
		if (direct)
			packed_lo = off;
	}
	if (off > packed_lo)
		HIP_TRY(hipMemcpyAsync(c->d_stage[s] + packed_lo, c->h_stage[s] + packed_lo, off - packed_lo,
				       hipMemcpyHostToDevice, c->s_copy[s]));
	HIP_TRY(hipMemcpyAsync(c->d_desc[s], c->h_desc[s], (size_t)m * sizeof(pech_desc), hipMemcpyHostToDevice,
			       c->s_copy[s]));
	HIP_TRY(hipEventRecord(c->ev_copied[s], c->s_copy[s]));
	HIP_TRY(hipStreamWaitEvent(c->s_comp, c->ev_copied[s], 0));
	int rc = ws_host_reserve(c, m);
	if (rc)
		return rc;
	rc = launch_batch(c, c->d_desc[s], c->d_out[s], m, c->d_ws_host, c->ws_host_bytes, c->s_comp, nullptr, nullptr,
			  nullptr, c->d_stat);
	if (rc)
		return rc;
	HIP_TRY(hipMemcpyAsync(c->h_out[s], c->d_out[s], (size_t)m * 4u, hipMemcpyDeviceToHost, c->s_comp));
	HIP_TRY(hipEventRecord(c->ev_done[s], c->s_comp));
	return 0;
}

// A single host buffer larger than a slot: chunk it and chain the register
// through the seed (crc32c(crc32c(s,A),B) == crc32c(s,A||B)).
static int host_big(DevCtx *c, const void *buf, size_t len, uint32_t seed, uint32_t *out, unsigned int flags)
{
	const uint8_t *p = (const uint8_t *)buf;
	uint32_t crc = seed;
	while (len) {
		const size_t m = len < c->stage_bytes ? len : c->stage_bytes;
		const void *b = p;
		const unsigned int l = (unsigned int)m;
		int rc = enqueue_host_slot(c, 0, &b, &l, nullptr, &crc, 0, 1, flags);
		if (rc)
			return rc;
		HIP_TRY(hipEventSynchronize(c->ev_done[0]));
		if ((rc = flat_check(c)))
			return rc;
		crc = c->h_out[0][0];
		p += m;
		len -= m;
	}
	*out = crc;
	return 0;
}

// Descriptors [i0, i0 + m) of one launch: at most STAGE_DESCS, and at most
// PECH_LAUNCH_MAX_BYTES of payload (the kernels count a launch's rows in
// 32 bits; only descriptors aliasing the same memory could exceed it).
static unsigned int launch_take(const unsigned int *lens, unsigned int i0, unsigned int end,
				unsigned int max_descs = STAGE_DESCS)
{
	uint64_t bytes = 0;
	unsigned int m = 0;
	while (i0 + m < end && m < max_descs && (m == 0 || bytes + lens[i0 + m] <= PECH_LAUNCH_MAX_BYTES))
		bytes += lens[i0 + m++];
	return m;
}

// CRC32C_F_PINNED | CRC32C_F_ALL_DEVICES: contiguous byte-balanced shards,
// one per device (PECH_DEVICES="0,0,..." overrides the list; up to
// PECH_MAX_SHARDS_PER_DEV shards per device share its two slots' descriptor
// space -- how the 1-GPU tests rehearse an 8-GPU split).
// Every shard's sub-batch is enqueued before any is waited for, so the GPUs
// read their host links concurrently from this one thread.
static int shard_pinned(const void *const *bufs, const unsigned int *lens, const uint32_t *seeds, uint32_t *out,
			unsigned int n, const int *devs, int nd);

// SURVEY 8(e), the optional split: a buffer larger than one device's fair
// share of the batch (and at least PECH_SPLIT_MIN_BYTES) is cut into
// per-device segments of whole 4 KiB pages, the first carrying the seed; the
// segment CRCs are combined on the host, R(s, A || B) = A_|B|(R(s, A)) ^
// R(0, B), so one huge buffer still keeps every GPU's host link busy.
#define PECH_SPLIT_MIN_BYTES (16u << 20)
#define PECH_MAX_SHARDS_PER_DEV 16
static int multi_device_pinned(const void *const *bufs, const unsigned int *lens, const uint32_t *seeds,
			       uint32_t *out, unsigned int n)
{
	int devs[64];
	const int nd = pech_internal_device_list(devs, 64, PECH_MAX_SHARDS_PER_DEV);
	if (nd < 0)
		return nd;
	uint64_t total = 0;
	for (unsigned int i = 0; i < n; ++i)
		total += lens[i];
	const uint64_t fair = total / (uint64_t)nd;
	bool split = false;
	for (unsigned int i = 0; i < n && nd > 1 && !split; ++i)
		split = lens[i] >= PECH_SPLIT_MIN_BYTES && lens[i] > fair;
	if (!split)
		return shard_pinned(bufs, lens, seeds, out, n, devs, nd);
	struct Seg {
		unsigned int orig;
		uint64_t after; // bytes of the buffer after this segment
	};
	std::vector<const void *> sb;
	std::vector<unsigned int> sl;
	std::vector<uint32_t> ss;
	std::vector<Seg> sg;
	for (unsigned int i = 0; i < n; ++i) {
		const uint32_t seed = seeds ? seeds[i] : 0u;
		unsigned int k = 1;
		if (lens[i] >= PECH_SPLIT_MIN_BYTES && lens[i] > fair)
			k = (unsigned int)std::min<uint64_t>((uint64_t)nd, (lens[i] + fair - 1) / std::max<uint64_t>(fair, 1));
		const uint64_t piece = ((uint64_t)lens[i] / k) & ~(uint64_t)4095;
		uint64_t off = 0;
		for (unsigned int j = 0; j < k; ++j) {
			const uint64_t len = j + 1 == k ? lens[i] - off : piece;
			sb.push_back((const char *)bufs[i] + off);
			sl.push_back((unsigned int)len);
			ss.push_back(j == 0 ? seed : 0u);
			sg.push_back(Seg{i, lens[i] - off - len});
			off += len;
		}
	}
	std::vector<uint32_t> so(sb.size());
	const int rc = shard_pinned(sb.data(), sl.data(), ss.data(), so.data(), (unsigned int)sb.size(), devs, nd);
	if (rc)
		return rc;
	for (unsigned int i = 0; i < n; ++i)
		out[i] = 0;
	for (size_t j = 0; j < sg.size(); ++j)
		out[sg[j].orig] ^= sg[j].after ? gf2_shift(so[j], sg[j].after) : so[j];
	return 0;
}

// Contiguous byte-balanced shards of the batch, one per listed device.
static int shard_pinned(const void *const *bufs, const unsigned int *lens, const uint32_t *seeds, uint32_t *out,
			unsigned int n, const int *devs, int nd)
{
	// shard k: slot slot[k] of its device, descriptors [off[k], off[k] + cap[k])
	// of it (one shard per device: the whole slot; u shards on one device
	// split the two slots' STAGE_DESCS between them; a device's shards share
	// its stream, so they run in order on one workspace)
	int slot[64], used[64] = {0}, nth[64];
	unsigned int off[64], cap[64];
	for (int k = 0; k < nd; ++k)
		nth[k] = used[devs[k]]++;
	for (int k = 0; k < nd; ++k) {
		const unsigned int per_slot = (unsigned int)(used[devs[k]] + 1) / 2u; // shards sharing one slot
		slot[k] = nth[k] & 1;
		cap[k] = STAGE_DESCS / per_slot;
		off[k] = (unsigned int)(nth[k] >> 1) * cap[k];
	}
	// shard k = buffers [cut[k], cut[k+1]): the first buffer whose byte prefix reaches k/nd of the total
	std::vector<uint64_t> pre(n + 1, 0);
	for (unsigned int i = 0; i < n; ++i)
		pre[i + 1] = pre[i] + lens[i];
	unsigned int cut[65];
	for (int k = 0; k <= nd; ++k) {
		const uint64_t target = (uint64_t)((__uint128_t)pre[n] * (unsigned)k / (unsigned)nd);
		cut[k] = k == nd ? n : (unsigned int)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
	}
	int cur = 0;
	HIP_TRY(hipGetDevice(&cur));
	struct Shard {
		DevCtx *c;
		unsigned int i0, m;
	} sh[64];
	int rc = 0;
	// device mappings of every buffer on its shard's device first: no launch if one is missing
	std::vector<uint64_t> dptr(n, 0);
	for (int k = 0; k < nd && !rc; ++k) {
		if ((rc = hipSetDevice(devs[k]) == hipSuccess ? 0 : -EIO))
			break;
		if ((rc = ctx_get(&sh[k].c)))
			break;
		if ((rc = stage_reserve(sh[k].c, sh[k].c->stage_bytes ? sh[k].c->stage_bytes : STAGE_BYTES, STAGE_DESCS)))
			break;
		if ((rc = ws_host_reserve(sh[k].c, STAGE_DESCS))) // before any launch: never regrown under one
			break;
		for (unsigned int i = cut[k]; i < cut[k + 1]; ++i) {
			void *dp = nullptr;
			if (lens[i] && (hipHostGetDevicePointer(&dp, const_cast<void *>(bufs[i]), 0) != hipSuccess || !dp)) {
				(void)hipGetLastError();
				set_err("crc32c_batch: buffer %u is not mapped on device %d (CRC32C_F_ALL_DEVICES)", i, devs[k]);
				rc = -EINVAL;
				break;
			}
			dptr[i] = (uint64_t)(uintptr_t)dp;
		}
		sh[k].i0 = cut[k];
	}
	for (bool more = !rc; more && !rc;) {
		more = false;
		for (int k = 0; k < nd && !rc; ++k) { // enqueue one sub-batch per shard
			Shard &S = sh[k];
			S.m = launch_take(lens, S.i0, cut[k + 1], cap[k]);
			if (!S.m)
				continue;
			DevCtx *c = S.c;
			const int s = slot[k];
			pech_desc *hd = c->h_desc[s] + off[k], *dd = c->d_desc[s] + off[k];
			uint32_t *ho = c->h_out[s] + off[k], *dout = c->d_out[s] + off[k];
			if ((rc = hipSetDevice(devs[k]) == hipSuccess ? 0 : -EIO))
				break;
			for (unsigned int j = 0; j < S.m; ++j) {
				const unsigned int i = S.i0 + j;
				hd[j].addr = dptr[i];
				hd[j].len = lens[i];
				hd[j].seed = seeds ? seeds[i] : 0u;
			}
			if (hipMemcpyAsync(dd, hd, (size_t)S.m * sizeof(pech_desc), hipMemcpyHostToDevice, c->s_comp) != hipSuccess) {
				set_err("hipMemcpyAsync: %s", hipGetErrorString(hipGetLastError()));
				rc = -EIO;
				break;
			}
			// shards on one device share its stream (ordered), so one workspace serves them
			if ((rc = launch_batch(c, dd, dout, S.m, c->d_ws_host, c->ws_host_bytes, c->s_comp, nullptr, nullptr,
					       nullptr, c->d_stat)))
				break;
			if (hipMemcpyAsync(ho, dout, (size_t)S.m * 4u, hipMemcpyDeviceToHost, c->s_comp) != hipSuccess) {
				set_err("hipMemcpyAsync: %s", hipGetErrorString(hipGetLastError()));
				rc = -EIO;
				break;
			}
		}
		for (int k = 0; k < nd && !rc; ++k) { // then wait for them all
			Shard &S = sh[k];
			if (!S.m)
				continue;
			if (hipSetDevice(devs[k]) != hipSuccess || hipStreamSynchronize(S.c->s_comp) != hipSuccess) {
				set_err("shard on device %d: %s", devs[k], hipGetErrorString(hipGetLastError()));
				rc = -EIO;
				break;
			}
			if ((rc = flat_check(S.c)))
				break;
			memcpy(out + S.i0, S.c->h_out[slot[k]] + off[k], (size_t)S.m * 4u);
			S.i0 += S.m;
			more = more || S.i0 < cut[k + 1];
		}
	}
	(void)hipSetDevice(cur);
	return rc;
}

static int host_batch(DevCtx *c, const void *const *bufs, const unsigned int *lens, const uint32_t *seeds,
		      uint32_t *out, unsigned int n, unsigned int flags)
{
	int rc = stage_reserve(c, STAGE_BYTES, STAGE_DESCS);
	if (rc)
		return rc;
	// slot bookkeeping for the double buffer
	unsigned int slot_i0[2] = {0, 0}, slot_m[2] = {0, 0};
	bool busy[2] = {false, false};
	int s = 0;
	unsigned int i = 0;
	auto drain = [&](int t) -> int {
		if (!busy[t])
			return 0;
		HIP_TRY(hipEventSynchronize(c->ev_done[t]));
		busy[t] = false;
		if (int e = flat_check(c))
			return e;
		memcpy(out + slot_i0[t], c->h_out[t], (size_t)slot_m[t] * 4u);
		return 0;
	};
	while (i < n) {
		if (lens[i] > c->stage_bytes) {
			for (int t = 0; t < 2; ++t)
				if ((rc = drain(t)))
					return rc;
			if ((rc = host_big(c, bufs[i], lens[i], seeds ? seeds[i] : 0u, &out[i], flags)))
				return rc;
			++i;
			continue;
		}
		// fill slot s with as many buffers as fit
		if ((rc = drain(s)))
			return rc;
		size_t bytes = 0;
		unsigned int m = 0;
		while (i + m < n && m < STAGE_DESCS && lens[i + m] <= c->stage_bytes) {
			const size_t nb = (bytes + lens[i + m] + 255u) & ~(size_t)255u;
			if (nb > c->stage_bytes)
				break;
			bytes = nb;
			++m;
		}
		if ((rc = enqueue_host_slot(c, s, bufs, lens, seeds, nullptr, i, m, flags)))
			return rc;
		slot_i0[s] = i;
		slot_m[s] = m;
		busy[s] = true;
		i += m;
		s ^= 1;
	}
	for (int t = 0; t < 2; ++t)
		if ((rc = drain(t)))
			return rc;
	return 0;
}

static int device_batch_sync(DevCtx *c, const void *const *bufs, const unsigned int *lens, const uint32_t *seeds,
			     uint32_t *out, unsigned int n)
{
	int rc = stage_reserve(c, c->stage_bytes ? c->stage_bytes : STAGE_BYTES, STAGE_DESCS);
	if (rc)
		return rc;
	for (unsigned int i0 = 0, m; i0 < n; i0 += m) {
		m = launch_take(lens, i0, n);
		for (unsigned int k = 0; k < m; ++k) {
			c->h_desc[0][k].addr = (uint64_t)(uintptr_t)bufs[i0 + k];
			c->h_desc[0][k].len = lens[i0 + k];
			c->h_desc[0][k].seed = seeds ? seeds[i0 + k] : 0u;
		}
		HIP_TRY(hipMemcpyAsync(c->d_desc[0], c->h_desc[0], (size_t)m * sizeof(pech_desc), hipMemcpyHostToDevice,
				       c->s_comp));
		if ((rc = ws_host_reserve(c, m)))
			return rc;
		if ((rc = launch_batch(c, c->d_desc[0], c->d_out[0], m, c->d_ws_host, c->ws_host_bytes, c->s_comp, nullptr,
				       nullptr, nullptr, c->d_stat)))
			return rc;
		HIP_TRY(hipMemcpyAsync(c->h_out[0], c->d_out[0], (size_t)m * 4u, hipMemcpyDeviceToHost, c->s_comp));
		HIP_TRY(hipStreamSynchronize(c->s_comp));
		if ((rc = flat_check(c)))
			return rc;
		memcpy(out + i0, c->h_out[0], (size_t)m * 4u);
	}
	return 0;
}

// ---------------------------------------------------------------------------
// drop-in routing, statistics, fault injection

// calls of at most this many bytes run on the host routine; PECH_CRC32C_CPU_MAX
// overrides the default, crc32c_set_cpu_max() changes it at run time
static const unsigned int CPU_MAX_DEFAULT = PECH_DROPIN_CPU_MAX_DEFAULT;
static std::atomic<unsigned int> g_cpu_max{CPU_MAX_DEFAULT};
static std::once_flag g_cpu_max_env;

static std::atomic<uint64_t> g_st_cpu_calls{0}, g_st_cpu_bytes{0}, g_st_gpu_calls{0}, g_st_gpu_bytes{0},
	g_st_fallbacks{0};
static std::atomic<int> g_fault[PECH_FAULT_SITES];

PECH_HIDDEN bool pech_fault(int site)
{
#ifndef PECH_TEST_HOOKS
	(void)site;
	return false; // release build: nothing can arm a fault
#endif
	if (site < 0 || site >= PECH_FAULT_SITES)
		return false;
	int v = g_fault[site].load(std::memory_order_relaxed);
	while (v > 0) {
		if (g_fault[site].compare_exchange_weak(v, v - 1))
			return v == 1;
	}
	return false;
}

static unsigned int cpu_max()
{
	std::call_once(g_cpu_max_env, [] {
		if (const char *e = getenv("PECH_CRC32C_CPU_MAX")) {
			char *end = nullptr;
			const unsigned long long v = strtoull(e, &end, 0);
			if (end != e)
				g_cpu_max.store(v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (unsigned int)v);
		}
	});
	return g_cpu_max.load(std::memory_order_relaxed);
}

// the GPU leg of the drop-in (runs on the library stack)
static int dropin_gpu(uint32_t crc, const void *data, unsigned int length, uint32_t *out)
{
	std::lock_guard<std::mutex> lk(g_mu);
	DevCtx *c = nullptr;
	int rc = ctx_get(&c);
	if (!rc)
		rc = stage_reserve(c, STAGE_BYTES, STAGE_DESCS);
	if (rc)
		return rc;
	if (pech_fault(PECH_FAULT_DROPIN_GPU)) {
		set_err("crc32c(): injected GPU failure (test)");
		return -EIO;
	}
	if (length > PECH_SMALL_MAX) {
		const void *b = data;
		const uint32_t s = crc;
		return host_batch(c, &b, &length, &s, out, 1, CRC32C_F_HOST);
	}
	// one launch: bytes into pinned staging, read there in place.  The
	// kernel writes the result, then this call's ticket, to pinned memory;
	// polling the ticket saves the stream synchronisation (~3 us).  After
	// ~20 ms of polling the stream is synchronised instead, which also
	// reports errors.
	memcpy(c->h_stage[0], data, length);
	const uint32_t ticket = ++c->small_ticket ? c->small_ticket : ++c->small_ticket;
	volatile uint32_t *res = (volatile uint32_t *)c->h_small;
	if (pech_launch_small(c->small_src, length, crc, c->d_consts, c->small_out, ticket, c->s_comp) != hipSuccess) {
		set_err("small-buffer launch: %s", hipGetErrorString(hipGetLastError()));
		return -EIO;
	}
	for (uint32_t spin = 0; res[1] != ticket && spin < (1u << 22); ++spin)
		__builtin_ia32_pause();
	if (res[1] != ticket && hipStreamSynchronize(c->s_comp) != hipSuccess) {
		set_err("small-buffer kernel: %s", hipGetErrorString(hipGetLastError()));
		return -EIO;
	}
	if (res[1] != ticket) {
		set_err("small-buffer kernel finished without its result");
		return -EIO;
	}
	*out = res[0];
	return 0;
}

// ---------------------------------------------------------------------------
// exported C-ABI
extern "C" {

uint32_t crc32c(uint32_t crc, const void *data, unsigned int length)
{
	if (length == 0)
		return crc; // include/crc32c.h:92: the loop body never runs
	if (length <= cpu_max()) {
		g_st_cpu_calls.fetch_add(1, std::memory_order_relaxed);
		g_st_cpu_bytes.fetch_add(length, std::memory_order_relaxed);
		return pech_cpu_crc32c(crc, data, length);
	}
	uint32_t out = 0;
	const int rc = on_lib_stack([&] { return dropin_gpu(crc, data, length, &out); });
	if (rc == 0) {
		g_st_gpu_calls.fetch_add(1, std::memory_order_relaxed);
		g_st_gpu_bytes.fetch_add(length, std::memory_order_relaxed);
		return out;
	}
	// total, like the reference: recompute on the host, report once
	if (g_st_fallbacks.fetch_add(1, std::memory_order_relaxed) == 0)
		fprintf(stderr, "pech_crc32c: crc32c() GPU path failed (%d: %s); computing on the CPU\n", rc, g_err);
	g_st_cpu_calls.fetch_add(1, std::memory_order_relaxed);
	g_st_cpu_bytes.fetch_add(length, std::memory_order_relaxed);
	return pech_cpu_crc32c(crc, data, length);
}

unsigned int crc32c_set_cpu_max(unsigned int bytes)
{
	(void)cpu_max(); // the environment is read first, so this call wins
	return g_cpu_max.exchange(bytes);
}

unsigned int crc32c_set_flat_max(unsigned int n)
{
	return g_flat_max.exchange(n < PECH_FLATG_MAX ? n : PECH_FLATG_MAX);
}

int crc32c_get_stats(struct crc32c_stats *st)
{
	if (!st) {
		set_err("crc32c_get_stats: null output");
		return -EINVAL;
	}
	st->cpu_calls = g_st_cpu_calls.load();
	st->cpu_bytes = g_st_cpu_bytes.load();
	st->gpu_calls = g_st_gpu_calls.load();
	st->gpu_bytes = g_st_gpu_bytes.load();
	st->gpu_fallbacks = g_st_fallbacks.load();
	// flat launches that reported a fault, on every initialised device (the
	// kernels count them: pech_flat_faults)
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		uint64_t faults = 0;
		st->gpu_faults = 0;
		bool any = false;
		for (int d = 0; d < 64; ++d)
			any = any || g_ctx[d].dev >= 0;
		if (!any)
			return 0; // (no GPU used: no HIP call)
		int cur = -1;
		if (hipGetDevice(&cur) != hipSuccess)
			cur = -1;
		for (int d = 0; d < 64; ++d) {
			if (g_ctx[d].dev < 0)
				continue;
			uint64_t v = 0;
			if (hipSetDevice(d) != hipSuccess || pech_read_flat_faults(&v)) {
				set_err("crc32c_get_stats: reading device %d's fault count failed", d);
				(void)hipGetLastError();
				continue;
			}
			faults += v;
		}
		if (cur >= 0)
			(void)hipSetDevice(cur);
		st->gpu_faults = faults;
		return 0;
	});
}

int crc32c_batch(const void *const *bufs, const unsigned int *lens, const uint32_t *seeds, uint32_t *out,
		 unsigned int n, unsigned int flags)
{
	if (n == 0)
		return 0;
	if (!bufs || !lens || !out || flags > (CRC32C_F_DEVICE | CRC32C_F_PINNED | CRC32C_F_ALL_DEVICES) ||
	    ((flags & CRC32C_F_DEVICE) && (flags & CRC32C_F_PINNED)) ||
	    ((flags & CRC32C_F_ALL_DEVICES) && !(flags & CRC32C_F_PINNED))) {
		set_err("crc32c_batch: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		if (flags & CRC32C_F_ALL_DEVICES)
			return multi_device_pinned(bufs, lens, seeds, out, n);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		if (flags & CRC32C_F_DEVICE)
			return device_batch_sync(c, bufs, lens, seeds, out, n);
		return host_batch(c, bufs, lens, seeds, out, n, flags);
	});
}

size_t crc32c_dev_workspace_bytes(unsigned int n)
{
	return ws_bytes_for(n < PECH_MAX_BATCH ? n : PECH_MAX_BATCH);
}

int crc32c_dev_batch_ws_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n, void *d_ws,
			      size_t ws_bytes, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_out || !d_ws) {
		set_err("crc32c_dev_batch_ws_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_batch(c, (const pech_desc *)d_descs, d_out, n, d_ws, ws_bytes, (hipStream_t)stream);
	});
}

int crc32c_dev_batch_small_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_out) {
		set_err("crc32c_dev_batch_small_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_small(c, (const pech_desc *)d_descs, d_out, n, (hipStream_t)stream);
	});
}

int crc32c_dev_reserve(unsigned int n)
{
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return ws_reserve(c, n);
	});
}

int crc32c_dev_batch_async(const struct crc32c_desc *d_descs, uint32_t *d_out, unsigned int n, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_out) {
		set_err("crc32c_dev_batch_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_internal_ws(c, (const pech_desc *)d_descs, d_out, n, (hipStream_t)stream, nullptr);
	});
}

int crc32c_dev_copy_batch_ws_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				   unsigned int n, void *d_ws, size_t ws_bytes, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_dsts || !d_out || !d_ws) {
		set_err("crc32c_dev_copy_batch_ws_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_batch(c, (const pech_desc *)d_descs, d_out, n, d_ws, ws_bytes, (hipStream_t)stream,
				    d_dsts);
	});
}

int crc32c_dev_copy_batch_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				unsigned int n, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_dsts || !d_out) {
		set_err("crc32c_dev_copy_batch_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_internal_ws(c, (const pech_desc *)d_descs, d_out, n, (hipStream_t)stream, d_dsts);
	});
}

int crc32c_dev_copy_batch_small_async(const struct crc32c_desc *d_descs, const uint64_t *d_dsts, uint32_t *d_out,
				      unsigned int n, void *stream)
{
	if (n == 0)
		return 0;
	if (!d_descs || !d_dsts || !d_out) {
		set_err("crc32c_dev_copy_batch_small_async: invalid arguments");
		return -EINVAL;
	}
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		int rc = ctx_get(&c);
		if (rc)
			return rc;
		return launch_small(c, (const pech_desc *)d_descs, d_out, n, (hipStream_t)stream, d_dsts);
	});
}

uint32_t crc32c_shift(uint32_t v, uint64_t nbytes)
{
	return gf2_shift(v, nbytes);
}

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
	return gf2_shift(crc_a, len_b) ^ crc_b;
}

// crc32c(seed, S_0 || ... || S_{n-1}) = A_L(seed) ^ XOR_i A_{after_i}(crc_i),
// folded left to right: acc <- A_|S_i|(acc) ^ crc_i (Horner over segments)
uint32_t crc32c_concat(uint32_t seed, const uint32_t *crcs, const uint64_t *lens, unsigned int n)
{
	uint32_t acc = seed;
	for (unsigned int i = 0; i < n; ++i)
		acc = gf2_shift(acc, lens[i]) ^ crcs[i];
	return acc;
}

int crc32c_device_init(void)
{
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		DevCtx *c = nullptr;
		return ctx_get(&c);
	});
}

int crc32c_timing(int enable)
{
	std::lock_guard<std::mutex> lk(g_mu);
	g_timing = enable != 0;
	return 0;
}

int crc32c_timing_read(double *kernel_ms, uint64_t *launches)
{
	return on_lib_stack([&] {
		std::lock_guard<std::mutex> lk(g_mu);
		double ms = 0;
		uint64_t cnt = 0;
		g_samples.clear();
		for (int d = 0; d < 64; ++d) {
			DevCtx *c = &g_ctx[d];
			for (auto &tl : c->pending) {
				HIP_TRY(hipEventSynchronize(tl.b));
				float t = 0;
				HIP_TRY(hipEventElapsedTime(&t, tl.a, tl.b));
				ms += t;
				++cnt;
				g_samples.push_back(t);
				c->free_events.push_back(tl);
			}
			c->pending.clear();
		}
		if (kernel_ms)
			*kernel_ms = ms;
		if (launches)
			*launches = cnt;
		return 0;
	});
}

int crc32c_timing_samples(float *ms, unsigned int max)
{
	std::lock_guard<std::mutex> lk(g_mu);
	if (!ms && max) {
		set_err("crc32c_timing_samples: null output");
		return -EINVAL;
	}
	const size_t k = g_samples.size() < max ? g_samples.size() : max;
	for (size_t i = 0; i < k; ++i)
		ms[i] = g_samples[i];
	return (int)g_samples.size();
}

const char *crc32c_last_error(void)
{
	return g_err;
}

const char *crc32c_version(void)
{
	return pech_kernel_tag();
}

// ---- test hooks; not in include/.  Failure injection exists only in the
// test build (build/lib_test.so, -DPECH_TEST_HOOKS, tests/test_faults.py):
// the release library cannot be made to fail on purpose.
#ifdef PECH_TEST_HOOKS
// arm fault `site` (enum pech_fault_site) to fire on its countdown-th use
int crc32c_test_inject(int site, int countdown)
{
	if (site < 0 || site >= PECH_FAULT_SITES)
		return -EINVAL;
	g_fault[site].store(countdown);
	return 0;
}

// Read-only diagnostics (tests/test_cpu_path.py), also test build only.
// the host routine itself: variant 0 = the one crc32c() uses (SSE4.2 when
// the CPU has it), 1 = portable slice-by-8
uint32_t crc32c_test_cpu(uint32_t crc, const void *data, size_t n, int variant)
{
	return variant ? pech_cpu_crc32c_portable(crc, data, n) : pech_cpu_crc32c(crc, data, n);
}

int crc32c_test_cpu_has_sse42(void)
{
	return pech_cpu_has_sse42();
}

// 1 if fn runs on the library stack when called through it (stack switch check)
int crc32c_test_stack_switch(void)
{
	return on_lib_stack([] { return pech_on_lib_stack(); });
}
#endif

} // extern "C"
