"""Build sanity of the gfx950 kernels (CPU: hipcc cross-compiles).

Guards two failure classes found on the GPU:
  * device helpers compiled as real calls (s_swappc) instead of being
    inlined -- a call in the plan kernel corrupted a live register across it;
  * the prefetch ring spilling to scratch or blowing the 128-VGPR budget that
    16 waves per CU (one 1024-thread workgroup) need.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "pech_amd", "csrc", "crc32c_kernels.hip")


@pytest.fixture(scope="module")
def device_asm():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    d = tempfile.mkdtemp()
    out = os.path.join(d, "k.s")
    # PECH_TEST_KFLAGS: extra -D flags, to hold an A/B variant to the same ISA checks
    extra = os.environ.get("PECH_TEST_KFLAGS", "").split()
    r = subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-Rpass-analysis=kernel-resource-usage", *extra, SRC, "-o", out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return open(out).read(), r.stderr


def kernel_body(asm, name):
    # the whole function: an early exit (an idle workgroup) may put an
    # s_endpgm before the row loops
    m = re.search(r"^%s:[^\n]*\n(.*?)^\.Lfunc_end" % name, asm, flags=re.S | re.M)
    assert m, name
    return m.group(1)


@pytest.mark.parametrize("kernel", ["pech_crc32c_plan", "pech_crc32c_main", "pech_crc32c_plan_copy",
                                    "pech_crc32c_main_copy", "pech_crc32c_small", "pech_crc32c_direct",
                                    "pech_crc32c_direct_copy", "pech_crc32c_flat", "pech_crc32c_flat_il",
                                    "pech_crc32c_flatg"])
def test_no_calls_no_scratch(device_asm, kernel):
    asm, _ = device_asm
    body = kernel_body(asm, kernel)
    assert "s_swappc" not in body and "s_setpc" not in body, "device helper not inlined"
    assert "scratch_" not in body and "buffer_store_dword" not in body, "register spill"


@pytest.mark.parametrize("kernel", ["pech_crc32c_main", "pech_crc32c_main_copy", "pech_crc32c_direct",
                                    "pech_crc32c_direct_copy", "pech_crc32c_flat", "pech_crc32c_flat_il",
                                    "pech_crc32c_flatg"])
def test_main_kernel_register_budget(device_asm, kernel):
    _, remarks = device_asm
    m = re.search(r"Function Name: %s \[.*?VGPRs: (\d+).*?ScratchSize \[bytes/lane\]: (\d+)" % kernel, remarks,
                  flags=re.S)
    assert m, remarks[-1000:]
    vgprs, scratch = int(m.group(1)), int(m.group(2))
    assert vgprs <= 128, f"{vgprs} VGPRs: 1024-thread workgroup would not fit one CU"
    assert scratch == 0


def test_main_kernel_hot_loop_shape(device_asm):
    asm, _ = device_asm
    body = kernel_body(asm, "pech_crc32c_main")
    # one v_perm per table lookup, lookups folded into ds_read offsets
    assert body.count("v_perm_b32") >= 16
    assert "ds_read_b32" in body and "offset:128" in body
    # the prefetch ring waits are counted, not drained
    assert re.search(r"s_waitcnt vmcnt\([1-9]\d*\)", body)
    # the five-operand XOR of a Horner step is two v_bitop3_b32
    assert "v_bitop3_b32" in body


def _blocks(body):
    out, cur = [], None
    for line in body.split("\n"):
        m = re.match(r"^(\.LBB\w+):(.*)", line)
        if m:
            cur = [m.group(1), [], m.group(2)]
            out.append(cur)
        elif cur is not None and line.strip() and not line.strip().startswith(";"):
            cur[1].append(line.strip())
    return out


@pytest.mark.parametrize("kernel", ["pech_crc32c_main", "pech_crc32c_direct", "pech_crc32c_flat", "pech_crc32c_flat_il",
                                    "pech_crc32c_flatg"])
def test_row_loops_never_drain_the_ring(device_asm, kernel):
    """The row loops (basic blocks with a full block of Horner steps and
    their prefetch loads) keep PECH_U-1 loads in flight across the back
    edge: no vmcnt(0) and no ring-register copies (which is what a ring
    slot holding two live values compiles to -- found in the ISA of v0.3)."""
    asm, _ = device_asm
    body = kernel_body(asm, kernel)
    # every block holding a run of Horner steps with their prefetch loads
    loops = [(n, ins) for n, ins, note in _blocks(body)
             if sum(i.startswith("v_perm_b32") for i in ins) >= 64
             and sum(i.startswith("global_load_dwordx4") for i in ins) >= 4]
    assert len(loops) >= 2, [(n, note) for n, _, note in _blocks(body)]
    for name, ins in loops:
        waits = [i for i in ins if "vmcnt(0)" in i]
        assert not waits, (name, waits)
        movs = [i for i in ins if i.startswith("v_mov_b32") or i.startswith("v_mov_b64")]
        assert len(movs) <= 8, (name, len(movs))


@pytest.mark.parametrize("kernel", ["pech_crc32c_main", "pech_crc32c_flat", "pech_crc32c_flatg", "pech_crc32c_direct"])
def test_row_loops_keep_lookups_in_flight(device_asm, kernel):
    """The hot row loop (the first block of Horner rows with prefetch loads)
    waits for its LDS lookups with counted lgkmcnt, several in flight.  A
    schedule that waits lgkmcnt(0) after every lookup pair ran flat launches
    4-5 us slower: the runtime interleave decision in pech_crc32c_flat (v0.33
    first build) and the scalar descriptor loads of flatg's small steps both
    produced it (profiles/r06/ab_flat_il_fix.txt, flatg.txt)."""
    asm, _ = device_asm
    loops = [(n, ins) for n, ins, note in _blocks(kernel_body(asm, kernel))
             if sum(i.startswith("v_perm_b32") for i in ins) >= 64
             and sum(i.startswith("global_load_dwordx4") for i in ins) >= 4]
    assert loops, kernel
    name, ins = loops[0]
    zero = sum("lgkmcnt(0)" in i for i in ins)
    assert zero <= 16, (name, zero)


def _loop_regions(body):
    """Every loop of a kernel body, from its "Loop Header" label to the last
    branch back to it (the fused-copy kernel's loops span several basic
    blocks): [(label, lines)]."""
    lines = body.split("\n")
    heads = []  # (line, label): the header comment sits on the label's line or the next one
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m and ("Loop Header" in l or (i + 1 < len(lines) and "Loop Header" in lines[i + 1]
                                         and not lines[i + 1].lstrip().startswith("."))):
            heads.append((i, m.group(1)))
    out = []
    for i0, label in heads:
        pat = re.compile(r"^\s*s_(?:cbranch_\w+|branch)\s+%s\b" % re.escape(label))
        back = [i for i, l in enumerate(lines) if i > i0 and pat.search(l)]
        if back:
            out.append((label, lines[i0:back[-1] + 1]))
    return out


@pytest.mark.parametrize("kernel", ["pech_crc32c_main", "pech_crc32c_flat", "pech_crc32c_flat_il", "pech_crc32c_flatg"])
def test_loops_with_ring_loads_never_wait_for_zero(device_asm, kernel):
    """Loop-level form of the check: every loop of the CRC kernel that issues
    ring loads has only counted vmcnt waits."""
    asm, _ = device_asm
    checked = 0
    for label, region in _loop_regions(kernel_body(asm, kernel)):
        if sum("global_load_dwordx4" in l for l in region) < 4:
            continue
        checked += 1
        assert not [l for l in region if "vmcnt(0)" in l], label
    assert checked >= 1, checked  # the step loop, which holds every row loop


def test_copy_row_loops_group_their_stores(device_asm):
    """The fused-copy kernel's block discipline (vmcnt counts stores and
    retires in issue order, so a store issued between two ring loads makes
    the later load's wait cover it): in each innermost row loop the stores
    come as one run, between the block's Horner rows and the next block's
    loads -- at most one load->store and one store->load switch per
    iteration, where the rotating ring had one per row."""
    asm, _ = device_asm
    U = int(re.search(r"#define PECH_U_COPY (\d+)", open(SRC).read()).group(1))
    rowloops = []
    for label, region in _loop_regions(kernel_body(asm, "pech_crc32c_main_copy")):
        ops = [("L" if "global_load_dwordx4" in l else "S") for l in region
               if "global_load_dwordx4" in l or "global_store_dwordx4" in l]
        if ops.count("L") >= U - 1 and ops.count("S") >= U and ops.count("L") <= 2 * U:
            rowloops.append((label, ops))
    assert len(rowloops) >= 2, [(lb, "".join(o)) for lb, o in rowloops]  # the full and the ragged block loops
    for label, ops in rowloops:
        switches = sum(a != b for a, b in zip(ops, ops[1:]))
        assert switches <= 2, (label, "".join(ops))


def _hipcc():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    return hipcc


@pytest.mark.parametrize("flag", ["-DPECH_AB_NOLDS", "-DPECH_AB_NOLOAD", "-DPECH_AB_NOATOMIC", "-DPECH_AB_NOSHIFT"])
def test_result_changing_switches_need_pech_diag(flag):
    # a stray diagnostic -D must not build a library that returns wrong CRCs
    r = subprocess.run([_hipcc(), "-E", "--offload-arch=gfx950", "--cuda-device-only", flag, SRC, "-o", os.devnull],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "PECH_DIAG" in r.stderr
    r = subprocess.run([_hipcc(), "-E", "--offload-arch=gfx950", "--cuda-device-only", flag, "-DPECH_DIAG", SRC,
                        "-o", os.devnull], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


def test_release_library_is_not_a_diagnostic_build():
    lib = os.path.join(REPO, "pech_amd", "libpech_crc32c.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    blob = open(lib, "rb").read()
    assert b"PECH OOB" not in blob          # not the bounds-checked build
    assert b"pech_stamps" not in blob       # not the stamps build
    assert b"pech_read_stamps" not in blob


def test_row_addr_launder_survives(device_asm):
    """row_addr() launders the row-0 address through an empty asm: without it
    LLVM folded ad + zoff back to ad for virtual leading pieces (a read
    before the buffer; a GPU fault at allocation starts in r01).  The launder
    shows as inline-asm markers in the main kernels' ISA, and each one's
    output feeds a ring load."""
    asm, _ = device_asm
    for kernel in ("pech_crc32c_main", "pech_crc32c_main_copy"):
        body = kernel_body(asm, kernel)
        n = body.count(";;#ASMSTART")
        assert n >= 4, (kernel, n)
        lines = [l.strip() for l in body.split("\n")]
        fed = 0
        for i, l in enumerate(lines):
            if l.startswith(";;#ASMEND"):
                nxt = lines[i + 1:i + 40]
                if any(x.startswith("global_load_dwordx4") for x in nxt):
                    fed += 1
        assert fed >= 4, (kernel, fed, n)


def test_no_comma_vector_casts():
    """`(u32x4)(a, b, c, d)` is a C++ comma expression: it splats `d`, it is
    not a vector literal (OpenCL's meaning).  v0.11's prologue wrote its
    per-chunk non-empty counts that way and plan_step then walked past the
    chunk (a GPU fault in the async tests).  Vector literals take braces."""
    pat = re.compile(r"\((?:u32x4|g_u32x4|uint4|u64x2)\)\s*\(([^()]|\([^()]*\))*,")
    for d in ("pech_amd/csrc", "tools"):
        for f in os.listdir(os.path.join(REPO, d)):
            if f.endswith((".hip", ".cpp", ".h")):
                src = open(os.path.join(REPO, d, f)).read()
                bad = [l for l in src.split("\n") if pat.search(l.split("//")[0])]
                assert not bad, (f, bad)
