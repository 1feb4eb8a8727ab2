"""Round-3 knobs: drain helper process and UVM residency defaults."""

from hipsnapshot import knobs



def test_arch_feature_parse():
    """XNACK mode comes from the device's arch-name feature suffixes."""
    assert knobs._arch_features("gfx950:sramecc+:xnack-") == {"sramecc": "+", "xnack": "-"}
    assert knobs._arch_features("gfx950") == {}


def test_round3_drain_and_uvm_knobs(monkeypatch):
    """Drain helper opt-in with bounded waits; never-placed UVM pages count as
    host-resident unless XNACK migrates them."""
    for k in ("HIPSNAPSHOT_DRAIN_PROCESS", "HIPSNAPSHOT_DRAIN_HELPER_MAP_TIMEOUT_S",
              "HIPSNAPSHOT_DRAIN_HELPER_TIMEOUT_S", "HIPSNAPSHOT_UVM_ASSUME_HOST"):
        monkeypatch.delenv(k, raising=False)
    assert knobs.drain_process() is False
    assert knobs.drain_helper_map_timeout_s() == 30.0
    assert knobs.drain_helper_timeout_s() == 1800.0
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: False)
    assert knobs.uvm_assume_host() is True
    # the device's own XNACK mode (not an environment variable) flips the default
    monkeypatch.setattr(knobs, "device_xnack_enabled", lambda index=0: True)
    assert knobs.uvm_assume_host() is False
    monkeypatch.setenv("HIPSNAPSHOT_UVM_ASSUME_HOST", "1")
    assert knobs.uvm_assume_host() is True
    monkeypatch.setenv("HIPSNAPSHOT_DRAIN_PROCESS", "1")
    monkeypatch.setenv("HIPSNAPSHOT_DRAIN_HELPER_MAP_TIMEOUT_S", "5")
    assert knobs.drain_process() is True and knobs.drain_helper_map_timeout_s() == 5.0
