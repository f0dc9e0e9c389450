"""Pin the oracle's evaluation and generation restatements (oracle.test_step_iw / estimate_log_prob_iw /
generate) against the reference's own outputs (tests/golden/make_golden.py eval: the reference's
TransformerVAE.sample with its KV cache, and test_step / estimate_log_prob_iw with injected draws). CPU only."""
import os

import numpy as np
import pytest
import torch

import oracle
from golden_util import GEN_NAMES, setup_gen, setup_iw


@pytest.mark.parametrize('name', GEN_NAMES)
def test_greedy_generation_matches_reference(name):
    torch.set_num_threads(min(8, os.cpu_count()))
    g, hp, params, z = setup_gen(name)
    T = int(g['cfg'][5])
    with torch.no_grad():
        out = oracle.generate(params, hp, z, T, int(g['start_token']), int(g['end_token']),
                              repetition_penalty=float(g['penalty']))
    np.testing.assert_array_equal(out.numpy(), g['tokens'])
    n = (g['tokens'] != 0).sum(1)
    assert n[0] < T - 2                             # row 0 stopped at the end token (early exit exercised)
    assert (n[1:] == T - 2).all()                   # the others ran to max_length (last slot stays 0)


def test_iw_nll_test_step_matches_reference():
    torch.set_num_threads(min(8, os.cpu_count()))
    g, hp, params, ids = setup_iw()
    with torch.no_grad():
        nll_iw = oracle.test_step_iw(params, hp, ids, torch.from_numpy(g['lens']), torch.from_numpy(g['eps_c1']),
                                     int(g['num_iter_c1']))
    assert abs(nll_iw.item() - float(g['nll_iw'])) <= 1e-5 * abs(float(g['nll_iw']))


def test_iw_chunked_broadcast_matches_reference():
    """chunk = B: the reference's [chunk, B, 1] + [chunk, B] broadcasting, reproduced shape for shape."""
    g, hp, params, ids = setup_iw()
    pad = ids.eq(0)
    with torch.no_grad():
        x = torch.nn.functional.embedding(ids, params['input_layer.0.weight'])
        enc = oracle.perceiver(params, x, pad, hp)
        mu, logvar, scale, _ = oracle.conditional_gaussian(params, enc)
        lp = oracle.estimate_log_prob_iw(params, hp, mu, scale, x, ids, pad, torch.from_numpy(g['eps_cB']),
                                         int(g['num_iter_cB']))
    assert lp.shape == g['log_prob_cB'].shape
    np.testing.assert_allclose(lp.numpy(), g['log_prob_cB'], rtol=1e-5)
