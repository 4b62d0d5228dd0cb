"""PluginSettings: the plugin's knobs read in one place (CPU)."""

from __future__ import annotations

import pytest

from distributed_learning_simulation_lib_amd import FedAVGAlgorithm
from distributed_learning_simulation_lib_amd.algorithm.dynamic_wave import DynamicWaveSettings, PluginSettings


def test_defaults_without_environment():
    s = PluginSettings.from_env({})
    assert s == PluginSettings()
    assert (s.wave_size, s.wave_min, s.eager_nan_check, s.qsgd_host_pointers) == (64, 0, False, True)
    assert s.dynamic == DynamicWaveSettings(enabled=True, batch=2, min_rows=4, idle_us=200, life_us=2_000_000)


def test_every_knob_from_the_environment():
    env = {"FEDAVG_WAVE_SIZE": "32", "FEDAVG_WAVE_MIN": "3", "FEDAVG_EAGER_NAN": "1", "FEDAVG_QSGD_HOST_PTRS": "0",
           "FEDAVG_DYN": "0", "FEDAVG_DYN_BATCH": "4", "FEDAVG_DYN_MIN_ROWS": "9", "FEDAVG_DYN_IDLE_US": "250",
           "FEDAVG_DYN_LIFE_US": "7000"}
    s = PluginSettings.from_env(env)
    assert (s.wave_size, s.wave_min, s.eager_nan_check, s.qsgd_host_pointers) == (32, 3, True, False)
    assert s.dynamic == DynamicWaveSettings(enabled=False, batch=4, min_rows=9, idle_us=250, life_us=7000)


def test_keyword_arguments_override_single_fields(monkeypatch):
    monkeypatch.setenv("FEDAVG_WAVE_SIZE", "16")
    monkeypatch.setenv("FEDAVG_DYN", "0")
    a = FedAVGAlgorithm(device="cpu")
    assert a.wave_size == 16 and a.dynamic_wave is False
    b = FedAVGAlgorithm(device="cpu", wave_size=8, dynamic_wave=True, eager_nan_check=True)
    assert (b.wave_size, b.dynamic_wave, b.eager_nan_check) == (8, True, True)
    assert b.settings.wave_size == 8 and b.settings.dynamic.enabled
    c = FedAVGAlgorithm(device="cpu", settings=PluginSettings(wave_size=5, dynamic=DynamicWaveSettings(idle_us=100)))
    assert c.wave_size == 5 and c.settings.dynamic.idle_us == 100 and c.dynamic_wave
    c.dynamic_wave = False
    assert not c.dynamic_wave and c.dyn_stats["open_failures"] == 0


@pytest.mark.parametrize("bad", [dict(wave_size=0), dict(wave_min=-1)])
def test_invalid_settings_are_refused(bad):
    with pytest.raises(ValueError):
        PluginSettings(**bad)
    with pytest.raises(ValueError):
        DynamicWaveSettings(batch=0)
