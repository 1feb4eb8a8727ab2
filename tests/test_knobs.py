"""UVM residency default: from the device's XNACK mode."""

from hipsnapshot import knobs


def test_arch_feature_parse():
    """XNACK mode comes from the device's arch-name feature suffixes."""
    assert knobs._arch_features("gfx950:sramecc+:xnack-") == {"sramecc": "+", "xnack": "-"}
    assert knobs._arch_features("gfx950") == {}


def test_uvm_assume_host_follows_device_xnack(monkeypatch):
    """Never-placed UVM pages count as host-resident unless the device's
    XNACK mode migrates them; ``TUNING.uvm_assume_host`` overrides."""
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: False)
    assert knobs.uvm_assume_host() is True
    # the device's own XNACK mode (not an environment variable) flips the default
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: True)
    assert knobs.uvm_assume_host() is False
    monkeypatch.setattr(knobs.TUNING, "uvm_assume_host", True)
    assert knobs.uvm_assume_host() is True


def test_env_surface_is_the_documented_table():
    """At most 25 HIPSNAPSHOT_* variables, every one the
    library reads is in ``knobs.ENV_KNOBS`` and documented in
    docs/getting_started.md."""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "hipsnapshot")
    used = set()
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip")):
                with open(os.path.join(dirpath, f), errors="replace") as fh:
                    used |= set(re.findall(r"HIPSNAPSHOT_([A-Z][A-Z0-9_]*[A-Z0-9])", fh.read()))
    assert len(knobs.ENV_KNOBS) <= 25
    assert used <= set(knobs.ENV_KNOBS), sorted(used - set(knobs.ENV_KNOBS))
    with open(os.path.join(root, "docs", "getting_started.md")) as fh:
        doc = fh.read()
    missing = [k for k in knobs.ENV_KNOBS if f"HIPSNAPSHOT_{k}" not in doc]
    assert not missing, missing


def test_plan_settings_ignore_tracing_and_threads(monkeypatch):
    """The plan caches' key holds the values plans depend on, not every
    environment variable."""
    base = knobs.plan_settings()
    monkeypatch.setenv("HIPSNAPSHOT_TIMELINE", "/tmp/x")
    monkeypatch.setenv("HIPSNAPSHOT_IO_THREADS", "3")
    assert knobs.plan_settings() == base
    monkeypatch.setenv("HIPSNAPSHOT_DISABLE_BATCHING", "1")
    assert knobs.plan_settings() != base
    with knobs.override_knob("RESTORE_SLOTS", 3):
        assert knobs.TUNING.restore_slots == 3
    assert knobs.TUNING.restore_slots == 6


def test_build_targets_gfx950_whatever_pytorch_rocm_arch_lists(monkeypatch):
    """the build took the first PYTORCH_ROCM_ARCH entry (often an
    older target on ROCm images); the kernels need gfx950."""
    import pytest

    from hipsnapshot import _build

    monkeypatch.setenv("PYTORCH_ROCM_ARCH", "gfx900;gfx906;gfx942")
    assert _build.gpu_archs() == ["gfx950"]
    monkeypatch.setenv("PYTORCH_ROCM_ARCH", "gfx90a;gfx950:xnack-")
    assert _build.gpu_archs() == ["gfx950:xnack-"]
    assert _build.gpu_archs("gfx950") == ["gfx950"]
    with pytest.raises(ValueError):
        _build.gpu_archs("gfx942")
