"""The C-ABI boundary on a machine without a GPU: the library loads, exports every entry
point include/mimo_engine.h declares, and validates configurations host-side with the
reference's error messages (no HIP call happens before the first compute call)."""
import ctypes
import os
import re

import numpy as np
import pytest

import _engine

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mimo_engine.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mimo_\w+)\s*\(", text)))


def test_header_and_binding_agree():
    names = declared_functions()
    assert len(names) >= 20
    assert sorted(_engine.SYMBOLS) == names


def test_library_exports_every_declared_symbol():
    lib = _engine.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.mimo_abi_version() == 8


def test_build_entry_checks_the_header_abi():
    """__graft_entry__.build() compares the library's ABI with include/mimo_engine.h's
    MIMO_ABI_VERSION (a hard-coded number there went stale once: ABI 5 -> 6)."""
    import __graft_entry__ as g
    assert g._header_abi_version() == _engine.lib().mimo_abi_version() == 8


def _cfg(**kw):
    tx = np.zeros((kw.get("n_ant", 4), 3))
    fr = np.full(kw.get("n_fft", 256), 3.5e9)
    base = dict(n_ant=4, n_sub_carr=128, n_fft=256, constel_size=16, cp_len=16, channel_kind=1, receiver_kind=1,
                device=-1, rx_loc_var=10.0, reroll_chan=1, precision=0)
    base.update(kw)
    c = _engine.MimoConfig(**base, tx_pos=tx.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           carrier_freqs=fr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return c, (tx, fr)


@pytest.mark.parametrize("kw,msg", [
    (dict(n_fft=300), "n_fft must be a power of two"),
    (dict(n_fft=16384), "n_fft must be a power of two"),
    (dict(n_sub_carr=256), "n_sub_carr must be a multiple of 4"),
    (dict(n_sub_carr=126), "n_sub_carr must be a multiple of 4"),
    (dict(constel_size=8), "only square QAM supported"),      # modulation.py:236-237
    (dict(constel_size=36), "only square QAM supported"),
    (dict(n_ant=0), "n_ant must be in"),
    (dict(channel_kind=7), "unknown channel_kind"),
    (dict(receiver_kind=0), "unknown receiver_kind"),
    (dict(precision=2), "precision must be"),
    (dict(chan_replay_period=-1), "chan_replay_period must be >= 0"),
    (dict(chan_replay_period=8, channel_kind=2), "Rayleigh channel only"),
])
def test_create_rejects_invalid_configs(kw, msg):
    lib = _engine.lib()
    c, keep = _cfg(**kw)
    h = lib.mimo_engine_create(ctypes.byref(c))
    assert not h
    assert msg in lib.mimo_last_error().decode()


def test_valid_engine_is_host_only_until_run():
    """create / set_point / describe / destroy never touch HIP (fork safety)."""
    lib = _engine.lib()
    c, keep = _cfg(n_fft=512, n_sub_carr=256)
    h = lib.mimo_engine_create(ctypes.byref(c))
    assert h
    pt = _engine.MimoPoint(ibo_db=3.0, snr_db=20.0, avg_symbol_power=10.0, pa_kind=1, cnc_pa_kind=1, sat_pow=1.0,
                           p_hardness=0.0, toi_coeff=0.0, cnc_sat_pow=1.0, cnc_toi_coeff=0.0, cnc_alpha=0.9,
                           csi_eps=-1.0)
    assert lib.mimo_engine_set_point(h, ctypes.byref(pt)) == 0
    desc = lib.mimo_engine_describe(h).decode()
    assert "F=512" in desc and "aligned" in desc and desc.endswith("f64"), desc
    bad = _engine.MimoPoint(**{f: getattr(pt, f) for f, _ in _engine.MimoPoint._fields_})
    bad.csi_eps = 1.5
    assert lib.mimo_engine_set_point(h, ctypes.byref(bad)) == -1  # MIMO_EINVAL
    assert "csi_eps" in lib.mimo_last_error().decode()
    lib.mimo_engine_destroy(h)


def test_set_point_array_alpha_validation():
    """mimo_point.array_alpha (ABI 8): 0 = per-antenna gains; > 0 accepted by the float64
    instances and by float32 up to F 4096; negative / non-finite values and float32 F 8192
    (no alpha polynomial in that instance) are MIMO_EINVAL -- all host-side, no HIP."""
    lib = _engine.lib()
    for prec, n_fft, alpha, ok in ((0, 512, 0.93, True), (1, 512, 0.93, True), (0, 8192, 0.93, True),
                                   (1, 8192, 0.93, False), (1, 8192, 0.0, True), (0, 512, -0.5, False),
                                   (0, 512, float("nan"), False), (0, 512, float("inf"), False)):
        c, keep = _cfg(n_fft=n_fft, n_sub_carr=n_fft // 2, precision=prec)
        h = lib.mimo_engine_create(ctypes.byref(c))
        assert h
        pt = _engine.Engine.make_point(3.0, 20.0, 10.0, "toi", toi_coeff=0.01, cnc_toi_coeff=0.01, cnc_alpha=0.9,
                                       array_alpha=alpha)
        rc = lib.mimo_engine_set_point(h, ctypes.byref(pt))
        assert (rc == 0) == ok, (prec, n_fft, alpha, rc, lib.mimo_last_error())
        if not ok:
            assert "array_alpha" in lib.mimo_last_error().decode()
        lib.mimo_engine_destroy(h)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_engine, "_lib", None)
    monkeypatch.setattr(_engine, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_engine.EngineError, match="not found"):
        _engine.lib()


def _engine_with_point():
    lib = _engine.lib()
    c, keep = _cfg(n_fft=512, n_sub_carr=256)
    h = lib.mimo_engine_create(ctypes.byref(c))
    pt = _engine.MimoPoint(ibo_db=3.0, snr_db=20.0, avg_symbol_power=10.0, pa_kind=1, cnc_pa_kind=1, sat_pow=1.0,
                           p_hardness=0.0, toi_coeff=0.0, cnc_sat_pow=1.0, cnc_toi_coeff=0.0, cnc_alpha=0.9,
                           csi_eps=-1.0)
    assert lib.mimo_engine_set_point(h, ctypes.byref(pt)) == 0
    return lib, h, pt, keep


@pytest.mark.parametrize("iters,first,n,msg", [
    ([2, 1], 0, 8, "sorted and unique"),
    ([1, 1], 0, 8, "sorted and unique"),
    ([32], 0, 8, "[0, 31]"),
    ([-1], 0, 8, "[0, 31]"),
    ([], 0, 8, "at least one iteration"),
    ([0], (1 << 32) - 4, 8, "fit 32 bits"),
])
def test_run_validates_arguments_before_any_hip_call(iters, first, n, msg):
    lib, h, pt, keep = _engine_with_point()
    it = np.asarray(iters, np.int32)
    err = np.zeros(4, np.uint64)
    bits = np.zeros(4, np.uint64)
    u64 = ctypes.POINTER(ctypes.c_uint64)
    rc = lib.mimo_engine_run(h, 1, first, n, it.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(it), 0,
                             err.ctypes.data_as(u64), bits.ctypes.data_as(u64), None)
    assert rc == -1 and msg in lib.mimo_last_error().decode()
    # before set_point
    c, keep2 = _cfg(n_fft=512, n_sub_carr=256)
    h2 = lib.mimo_engine_create(ctypes.byref(c))
    it0 = np.zeros(1, np.int32)
    rc = lib.mimo_engine_run(h2, 1, 0, 8, it0.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 1, 0,
                             err.ctypes.data_as(u64), bits.ctypes.data_as(u64), None)
    assert rc == -1 and "set_point" in lib.mimo_last_error().decode()
    lib.mimo_engine_destroy(h)
    lib.mimo_engine_destroy(h2)


@pytest.mark.parametrize("prec,team", [(0, 64), (1, 64)])
def test_precision_selects_the_instance(prec, team):
    """precision = MIMO_PREC_F64 (default 0: the reference's float64) or MIMO_PREC_F32."""
    lib = _engine.lib()
    c, keep = _cfg(n_fft=2048, n_sub_carr=1024, precision=prec)
    h = lib.mimo_engine_create(ctypes.byref(c))
    desc = lib.mimo_engine_describe(h).decode()
    # fp64 teams hold 8 points per thread (T = F/8), fp32 teams 16 (T = F/16)
    assert desc.startswith("F=2048 T=256" if prec == 0 else "F=2048 T=128"), desc
    assert desc.endswith("f64" if prec == 0 else "f32"), desc
    lib.mimo_engine_destroy(h)


def test_calc_alpha_validates_without_a_gpu():
    """mimo_calc_alpha (ABI 6): an empty request succeeds and a negative count is rejected
    host-side, before any HIP call."""
    lib = _engine.lib()
    out = np.zeros(1)
    dp = ctypes.POINTER(ctypes.c_double)
    assert lib.mimo_calc_alpha(out.ctypes.data_as(dp), 0, out.ctypes.data_as(dp)) == 0
    assert lib.mimo_calc_alpha(out.ctypes.data_as(dp), -1, out.ctypes.data_as(dp)) == -1  # MIMO_EINVAL
    assert "n < 0" in lib.mimo_last_error().decode()


def test_stale_library_reports_its_abi(tmp_path, monkeypatch):
    """a library of an older ABI (here 6, without mimo_cnc_receive_ex) is reported
    as such -- the version is checked before the newer entry points are bound, so the error
    is the 'rebuild it' EngineError, not a bare AttributeError."""
    import shutil
    import subprocess
    import _engine
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    src = tmp_path / "stale.c"
    src.write_text("int mimo_abi_version(void) { return 6; }\n")
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    monkeypatch.setattr(_engine, "_lib", None)
    monkeypatch.setattr(_engine, "LIB_PATH", str(so))
    with pytest.raises(_engine.EngineError, match="is ABI 6, this module ABI 8: rebuild it"):
        _engine.lib()
