"""Golden vectors for the sweep layer, from the REFERENCE itself (survey container only).

    python tests/golden/make_sweep_golden.py  [--ref /root/reference]

Records, as JSON data in tests/golden/sweep_golden.json:
  * the parsed reference default config (config/default_config.yaml),
  * generate_param_combinations(config, type) for all four experiment types,
    on the default config and on a config with state_representation lists,
  * get_model_params(config) and with overrides,
  * get_folder_name(...) for a set of parameter tuples (src/experiments/runner.py:11-45).
The reference's runner module imports SPGG (and h5py at module top): an
in-memory h5py stand-in is installed first, as in make_golden.py.
"""
import argparse
import copy
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))

TUPLES = [
    (3.6, 0.0, False, 0.8, 1.0, 1.0, "reputation", "qlearning"),
    (3.6, 0.5, True, 0.8, 1.0, 1.0, "action", "sarsa"),
    (3.0, 1.0, True, 0.8, 0.95, 1.0, "reputation", "double_qlearning"),
    (1.0, 2.0, False, 0.1, 0.83, 0.5, "action", "expected_sarsa"),
    (5, 1, True, 0.8, 0.833333, 1.25, "reputation", "qlearning"),
    (2.25, 0.0, False, 0.8, 1, 1, "reputation", "qlearning"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    import matplotlib
    matplotlib.use("Agg")
    sys.modules["h5py"] = types.SimpleNamespace(File=None)
    sys.path.insert(0, args.ref)
    from src.config_loader import load_config, generate_param_combinations, get_model_params
    from src.experiments.runner import get_folder_name
    cfg = load_config(None)
    cfg2 = copy.deepcopy(cfg)
    cfg2["rl"]["state_representation"] = "action"
    cfg2["experiments"]["figure_2_3_4"]["state_representation"] = ["reputation", "action"]
    cfg2["experiments"]["custom"]["state_representation"] = "action"
    cfg2["experiments"]["custom"]["r_values"] = [3.0, 3.0, 2.5]
    out = {"default_config": cfg, "combos": {}, "combos_states": {}}
    for t in ("figure_2_3_4", "figure_6_7_8_9", "all_figures", "custom"):
        out["combos"][t] = [list(x) for x in generate_param_combinations(cfg, t)]
        out["combos_states"][t] = [list(x) for x in generate_param_combinations(cfg2, t)]
    out["config_states"] = cfg2
    out["model_params"] = get_model_params(cfg)
    out["model_params_over"] = get_model_params(cfg, L=64, iterations=10, algorithm="sarsa")
    out["model_params_empty"] = get_model_params({})
    out["folders"] = [[list(t), get_folder_name(*t)] for t in TUPLES]
    out["folders7"] = [[list(t[:7]), get_folder_name(*t[:7])] for t in TUPLES]
    with open(os.path.join(HERE, "sweep_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote sweep_golden.json")


if __name__ == "__main__":
    main()
