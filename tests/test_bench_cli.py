"""bench.py's host-side logic on CPU (no GPU): the config table, the algorithmic byte model and the
CPU-baseline worker of every config (config 5: the 16-bit oracle path)."""
import importlib.util
import os
import subprocess
import sys

import pytest

from jmpaths import ensure_built

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_config_table():
    b = load_bench()
    c = b.use_config(2)
    assert (b.W, b.H, b.BD, b.BYTES_PER_PIXEL, c["search_mode"]) == (1920, 1088, 8, 9.0, 0)
    c = b.use_config(5)
    assert (b.W, b.H, b.BD, c["slice_mbs"], c["t8"], c["search_mode"], b.RDO) == (3840, 2160, 10, 240, 0, 3, 1)
    assert b.BYTES_PER_PIXEL == 15.0   # four 16-bit picture terms + int16 levels
    c = b.use_config(5, rdo=0)          # the RDO-off variant of config 5's shape
    assert (c["t8"], b.RDO) == (1, 0) and "RDO off" in c["metric"]
    c = b.use_config(3)
    assert (b.BD, b.BYTES_PER_PIXEL) == (8, 9.0)


@pytest.mark.parametrize("config,mode,rdo", [(2, 0, 0), (3, 3, 0), (5, 3, 1), (5, 3, 0)])
def test_cpu_worker(config, mode, rdo, tmp_path):
    """the cpu_baseline child on a small picture: prints its seconds; config 5 dumps 16-bit recon
    (RDO on: the oracle's RD loop; its MBs carry their CABAC rates in min_cost)"""
    ensure_built()
    dump = tmp_path / "d.npz"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-worker", "0", str(config), str(mode), "64x48",
                        str(dump)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, JMH_BENCH_SLICE_MBS="4" if config == 5 else "0", JMH_BENCH_RDO=str(rdo)))
    assert r.returncode == 0, r.stderr
    assert float(r.stdout.split()[-1]) > 0
    import numpy as np
    d = np.load(dump)
    assert d["py"].dtype == (np.uint16 if config == 5 else np.uint8)
    if config == 5:
        assert int(d["py"].max()) > 255
    if rdo:
        assert d["pres"]["min_cost"].sum() > 0


def test_exit_status():
    """an incomplete timed region is its own failure (4), never reported as an oracle mismatch (3);
    `verified` None (no oracle leg) with a complete region is success"""
    b = load_bench()
    assert b.exit_status(True, True) == (0, None)
    assert b.exit_status(None, True) == (0, None)
    rc, msg = b.exit_status(None, False)
    assert rc == 4 and "oracle" not in msg and "--steps" in msg
    rc, msg = b.exit_status(True, False)
    assert rc == 4 and "oracle" not in msg
    rc, msg = b.exit_status(False, True)
    assert rc == 3 and "differ from the oracle" in msg
    assert b.exit_status(False, False)[0] == 3


def test_metric_names_timer():
    """every bench metric says which timer `value` uses (device-resident; the PCIe-inclusive rate
    is host_path.pcie_inclusive_mp_s)"""
    b = load_bench()
    for k in (2, 3, 5):
        assert "device-resident" in b.use_config(k)["metric"]
    assert "device-resident" in b.use_config(5, rdo=0)["metric"]


def test_pmc_records_issue_roofline():
    """tools/pmc_traffic.json carries the VALU instructions per MB the issue roofline of every
    config prices (configs 3 and 5 report bound "valu-issue")"""
    b = load_bench()
    b.use_config(3)
    for config, mode, t8, sl in ((2, 0, 0, 0), (3, 3, 1, 0), (5, 3, 0, 240), (5, 3, 1, 240)):
        b.RDO = 1 if config == 5 else 0
        rec, src = b.read_pmc_traffic(config, mode, t8, sl)
        assert rec and rec["valu_insts_per_mb"] > 4225 and rec["hbm_bytes_per_mb"] > 0, (config, src)
        assert abs(sum(rec["valu_kernels"].values()) - rec["valu_insts_per_mb"]) < 1


def test_available_cores():
    """all_cores runs one oracle process per core this process may use: its affinity mask, capped
    by a cgroup CPU quota where one is set (not a fixed 16)."""
    b = load_bench()
    n, aff, quota, online = b.available_cores()
    assert n == (aff if quota is None else max(1, min(aff, int(quota))))
    assert 1 <= n <= aff <= (online or aff)


def test_metric_names_search_override():
    """--search-mode names the measured search in the metric (config 2's metric says
    FullSearch for its FFS default; an EPZS override must not keep that name)."""
    import re
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'metric_sm="FullSearch"' in src
    b = load_bench()
    m = b.CONFIGS[2]["metric"]
    own = b.CONFIGS[2]["metric_sm"]
    assert own in m
    for sm, label in ((3, "EPZS"), (-1, "FullSearch SearchMode=-1")):
        got = m.replace(own, {0: "FFS", -1: "FullSearch SearchMode=-1", 3: "EPZS"}[sm], 1)
        assert label in got and re.search(r"@1080p " + re.escape(label) + " SR=32", got)
