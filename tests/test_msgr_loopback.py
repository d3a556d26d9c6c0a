"""The patched reference messenger itself, running:
build/msgr_loopback (tests/c/msgr_loopback.c, built by `make` in the build
container from temp patched copies of pech's sources, tests/pech_build.py)
starts pech's runtime as src/main.c does, opens a connection between two
ceph_messengers on 127.0.0.1 through a relay that can flip a bit on the
wire, and carries OSD_OP / OSD_OPREPLY messages with 0 B - 4 MiB data both
ways through the real read_partial_message / write_partial_message_data /
con_fault / ceph_msg_revoke paths.  Each scenario's own checks are in the
binary (its header); it prints one JSON line and exits 0 iff they hold.

* not gpu: no GPU in the build container, so the patch's async context is
  NULL and every connection checksums inline -- the reference's own path,
  through the same binary;
* gpu: the adapter's route (--expect-gpu: GPU submissions on both sides,
  none with NO_DATA_CRC, the corrupted payload caught as rx_bad), with the
  adapter's host cutoff at its default (8 KiB) and at 0 (every checked
  payload on the GPU)."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "msgr_loopback")
SCENARIOS = ["basic", "nocrc", "corrupt-req", "corrupt-reply", "revoke"]


def run(scenario, *args, env=None, timeout=150):
    assert os.path.exists(EXE), "build/msgr_loopback is built by `make` in the build container"
    # The revoke scenario is deterministic: the harness holds
    # the target's send in place until the revoke lands -- inline, its data
    # writes report a full socket while it is con->out_msg; with the adapter,
    # complete() delivers nothing while it is con->out_msg, so its footer is
    # held for the GPU CRC and revoked there (tests/c/msgr_loopback.c,
    # lb_holding).  One run, no retry.
    r = subprocess.run([EXE, scenario, *args], capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    res = {}
    for l in lines:  # the contexts' counters, then the scenario's line
        res.update(json.loads(l))
    assert r.returncode == 0 and res["ok"], json.dumps(res) + "\n" + r.stderr[-3000:]
    return res


def common(res):
    assert res["unanswered"] == 0 and res["msgs_alloc"] == res["msgs_freed"]
    for k in ("bad_bytes", "bad_footer", "bad_order", "bad_front"):
        assert res[k] == 0, k
    if res["scenario"] in ("corrupt-req", "corrupt-reply"):
        assert res["relay_flips"] == 1 and res["relay_conns"] >= 2 and res["cli_faults"] >= 1
    if res["scenario"] == "revoke":
        assert res["revoked_mid_send"] == 1 and res["srv_dispatched"] - res["srv_dups"] == res["requests"] - 2
        # the send was held until the revoke: its data writes (inline) or
        # its footer (adapter)
        assert res["held_writes"] >= 1 or res["revoked_footer_held"] == 1, res
    if res["scenario"] in ("basic", "nocrc"):
        assert res["srv_dups"] == 0 and res["cli_dups"] == 0 and res["cli_faults"] == 0
        assert res["srv_dispatched"] == res["cli_dispatched"] == res["requests"]


@pytest.mark.skipif(not os.path.exists(EXE) and not os.path.isdir("/root/reference/src"),
                    reason="built in the build container")
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_loopback_inline_crc(scenario):
    # the build container has no GPU: crc_ctx is NULL, the reference's path
    res = run(scenario)
    common(res)
    if not os.path.exists("/dev/kfd"):
        assert res["adapter"]["rx_submitted"] == res["adapter"]["tx_submitted"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_loopback_gpu_two_contexts(scenario):
    """One async context per entry of PECH_DEVICES (the patch
    spreads its connections over every GPU): "0,0" puts two on this box's
    GPU, and the client's and the server's connections land on different
    ones -- each context takes submissions, each connection's CRCs stay in
    order in its own."""
    res = run(scenario, "--expect-gpu", "--expect-contexts", "2", env={"PECH_DEVICES": "0,0"})
    common(res)
    assert len(res["contexts"]) == 2
    for c in res["contexts"]:
        assert c["device"] == 0 and (c["submitted"] == 0 if scenario == "nocrc" else c["submitted"] > 0), c


@pytest.mark.gpu
@pytest.mark.parametrize("host_max", [None, "0"])
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_loopback_gpu(scenario, host_max):
    env = {} if host_max is None else {"PECH_CRC32C_MSGR_HOST_MAX": host_max}
    res = run(scenario, "--expect-gpu", env=env)
    common(res)
    a = res["adapter"]
    if scenario != "nocrc":
        assert a["rx_submitted"] > 0 and a["tx_submitted"] > 0
        if host_max == "0":
            assert a["rx_host"] == 0 and a["tx_host"] == 0
    else:
        assert a["rx_submitted"] == a["tx_submitted"] == 0
    if scenario.startswith("corrupt"):
        assert a["rx_bad"] == 1
    if scenario == "revoke":  # revoked while its footer waited for the GPU CRC
        assert res["revoked_footer_held"] == 1 and a["tx_released"] >= 1
