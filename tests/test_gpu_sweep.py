"""Batched sweep runner on the MI355X: every experiment of a mixed batch writes,
into its reference-named folder, exactly the datasets the oracle (pinned to the
reference by the golden fixtures) produces for the same seed -- integer data
and the state bit-exact, device-reduced float histories within rtol 1e-5."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd import sweep  # noqa: E402
from spgg_amd.h5io import read_datasets  # noqa: E402
from oracle import spgg_oracle as O  # noqa: E402
from tests.test_gpu_parity import APPROX, FLOAT_TOL  # noqa: E402

SMALL = dict(L=16, iterations=60)
TUPLES = [
    (3.6, 1.0, False, 0.8, 1.0, 1.0, "reputation", "qlearning"),
    (3.0, 0.5, True, 0.8, 0.95, 1.0, "action", "sarsa"),
    (4.0, 1.0, False, 0.8, 0.95, 1.0, "reputation", "qlearning"),  # same batch as the first
    (3.6, 0.0, True, 0.8, 1.0, 1.0, "reputation", "double_qlearning"),
    (2.5, 1.0, False, 0.8, 0.95, 1.0, "action", "expected_sarsa"),
]
SEEDS = [11, 12, 13, 14, 15]


def _oracle(p8, seed):
    r, kappa, so, alpha, w_p, gain, state, alg = p8
    kw = dict(sweep.RUNNER_MODEL, **SMALL)
    op = O.Params(L=kw["L"], iterations=kw["iterations"], r=r, c=kw["c"], cost=kw["cost"], alpha=alpha,
                  gamma=kw["gamma"], epsilon=kw["epsilon"], epsilon_decay=kw["epsilon_decay"],
                  epsilon_min=kw["epsilon_min"], influence_factor=kappa, use_second_order=so,
                  lambda_epsilon=kw["lambda_epsilon"], delta_R_D=kw["delta_R_D"], R_min=kw["R_min"],
                  R_max=kw["R_max"], reward_weight_payoff=w_p, rep_gain_C=gain,
                  state_representation=state, algorithm=alg)
    return O.run(op, np.random.RandomState(seed), collect_snapshots=True)


def test_batched_sweep_matches_oracle(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    res = sweep.run_experiments(TUPLES, use_progress_bar=False, seeds=SEEDS, devices=[0],
                                save_png=False, **SMALL)
    assert [r[0] for r in res] == TUPLES          # input order, reference's return shape
    for p8, seed, (_, (coop, rep_mean)) in zip(TUPLES, SEEDS, res):
        folder = tmp_path / sweep.get_folder_name(*p8)
        for sub in ("configurations", "reputations", "plots/snapshots", "data"):
            assert (folder / sub).is_dir()
        got = read_datasets(str(folder / "data" / "experiment_data.h5"))
        ds, fin = _oracle(p8, seed)
        assert set(got) == set(ds), sorted(set(got) ^ set(ds))
        for k, w in ds.items():
            g = np.asarray(got[k])
            w = np.asarray(w)
            assert g.shape == w.shape, (k, g.shape, w.shape)
            if k in APPROX:
                np.testing.assert_allclose(g, w, equal_nan=True, err_msg=k, **FLOAT_TOL)
            else:
                assert np.array_equal(g, w, equal_nan=w.dtype.kind == "f"), k
        assert coop == float(np.sum(fin["S"] == 0)) / fin["S"].size
        assert rep_mean == 0


def test_run_one_experiment_dropin(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    p7 = (3.0, 1.0, False, 0.8, 0.95, 1.0, "reputation")
    params, (coop, rep_mean) = sweep.run_one_experiment(p7, **SMALL)
    assert params == p7 and 0.0 <= coop <= 1.0 and rep_mean == 0
    fn = tmp_path / sweep.get_folder_name(*p7) / "data" / "experiment_data.h5"
    assert "coop_rate_history" in read_datasets(str(fn))


def test_figures_regenerate_from_gpu_sweep(tmp_path, monkeypatch):
    """SURVEY §8f rank 4 end to end: the reference's paper-figure grid
    (all_figures + the state comparison pair) swept on the GPU, then every
    figure of scripts/plot_figures.py / plot_state_comparison.py regenerated
    from the files the sweep wrote."""
    from spgg_amd import figures
    monkeypatch.chdir(tmp_path)
    tuples = sweep.generate_param_combinations(sweep.DEFAULT_CONFIG, "all_figures")
    tuples += [(4.6, 0.0, False, 0.8, 1.0, 1.0, st) for st in ("reputation", "action")]
    small = dict(L=16, iterations=120)
    res = sweep.run_experiments(tuples, use_progress_bar=False, seeds=list(range(len(tuples))),
                                devices=[0], save_png=False, **small)
    assert len(res) == len(tuples)
    out = figures.plot_figures(str(tmp_path), str(tmp_path / "figs"), ["all"], total_iterations=120)
    assert sorted(out) == list(figures.FIGURES)
    for path in out.values():
        assert os.path.getsize(path) > 1000, path
    sc = figures.state_comparison(str(tmp_path), str(tmp_path / "figs"), total_iterations=121)
    assert os.path.getsize(sc) > 1000
    # every curve of Figure 2 is a file's coop_rate_history
    for k, paths in figures.figure_inputs(str(tmp_path))["2"].items():
        for p in paths.values():
            h = figures.load_data(p, "coop_rate_history")
            assert h is not None and 1 <= len(h) <= 120 and np.all((h >= 0) & (h <= 1))
