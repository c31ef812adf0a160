"""Sweep layer (spgg_amd.sweep) against the reference's own config loader and
runner naming, pinned by tests/golden/sweep_golden.json (make_sweep_golden.py
ran the reference's src/config_loader.py and src/experiments/runner.py)."""
import json
import os

import pytest

from spgg_amd import sweep

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "sweep_golden.json")))


def test_default_config_matches_reference_yaml():
    assert sweep.load_config(None) == GOLD["default_config"]


@pytest.mark.parametrize("etype", sweep.EXPERIMENT_TYPES)
def test_param_combinations_match_reference(etype):
    got = [list(x) for x in sweep.generate_param_combinations(sweep.load_config(), etype)]
    assert got == GOLD["combos"][etype]
    got2 = [list(x) for x in sweep.generate_param_combinations(GOLD["config_states"], etype)]
    assert got2 == GOLD["combos_states"][etype]


def test_unknown_experiment_type_raises():
    with pytest.raises(ValueError):
        sweep.generate_param_combinations(sweep.load_config(), "figure_5")


def test_model_params_match_reference():
    cfg = sweep.load_config()
    assert sweep.get_model_params(cfg) == GOLD["model_params"]
    assert list(sweep.get_model_params(cfg)) == list(GOLD["model_params"])  # key order too
    assert sweep.get_model_params(cfg, L=64, iterations=10, algorithm="sarsa") == GOLD["model_params_over"]
    assert sweep.get_model_params({}) == GOLD["model_params_empty"]


def test_folder_names_match_reference():
    for t, name in GOLD["folders"]:
        assert sweep.get_folder_name(*t) == name
    for t, name in GOLD["folders7"]:
        assert sweep.get_folder_name(*t) == name


def test_unpack_forms():
    t8 = (3.0, 1.0, True, 0.8, 0.95, 1.0, "action", "sarsa")
    assert sweep.unpack(t8) == t8
    assert sweep.unpack(t8[:7]) == t8[:7] + ("qlearning",)
    assert sweep.unpack(t8[:6]) == t8[:6] + ("reputation", "qlearning")
    with pytest.raises(ValueError):
        sweep.unpack(t8[:5])


def test_resolve_algorithms():
    cfg = sweep.load_config()
    assert sweep.resolve_algorithms(None, cfg) == ["qlearning"]
    assert sweep.resolve_algorithms(["all"], cfg) == list(sweep.ALGORITHMS)
    assert sweep.resolve_algorithms(["sarsa", "QLearning", "sarsa"], cfg) == ["qlearning", "sarsa"]
    with pytest.raises(ValueError):
        sweep.resolve_algorithms(["ppo"], cfg)


def test_load_config_yaml_roundtrip(tmp_path):
    import yaml
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump(GOLD["config_states"]))
    assert sweep.load_config(str(p)) == GOLD["config_states"]
    with pytest.raises(FileNotFoundError):
        sweep.load_config(str(tmp_path / "missing.yaml"))


def test_make_folders(tmp_path):
    f = str(tmp_path / sweep.get_folder_name(3.0, 1.0, False, 0.8, 1.0, 1.0))
    sweep.make_folders(f)
    for sub in ("configurations", "reputations", "plots", "plots/snapshots", "data"):
        assert os.path.isdir(os.path.join(f, sub))
