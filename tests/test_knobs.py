"""UVM residency default: from the device's XNACK mode."""

from hipsnapshot import knobs


def test_arch_feature_parse():
    """XNACK mode comes from the device's arch-name feature suffixes."""
    assert knobs._arch_features("gfx950:sramecc+:xnack-") == {"sramecc": "+", "xnack": "-"}
    assert knobs._arch_features("gfx950") == {}


def test_uvm_assume_host_follows_device_xnack(monkeypatch):
    """Never-placed UVM pages count as host-resident unless the device's
    XNACK mode migrates them; the env knob overrides."""
    monkeypatch.delenv("HIPSNAPSHOT_UVM_ASSUME_HOST", raising=False)
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: False)
    assert knobs.uvm_assume_host() is True
    # the device's own XNACK mode (not an environment variable) flips the default
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: True)
    assert knobs.uvm_assume_host() is False
    monkeypatch.setenv("HIPSNAPSHOT_UVM_ASSUME_HOST", "1")
    assert knobs.uvm_assume_host() is True
