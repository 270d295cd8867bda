"""The cluster LSTM recurrences' selectable hand-off forms (csrc/lstm_coop.hip; the
reference's nn.LSTM of src/model.py:16-22, 38-41) are the same arithmetic: every
form must give the default form's outputs bit for bit, and each form must
reproduce itself call after call (the round-4 store hazard showed up as exactly
such a run-to-run difference).

  forward:  IRC_LSTM_COOP_SENTINELS=1 (wave-0 sentinel pass before the sweep),
            IRC_LSTM_COOP_WAVE_PUBLISH=0 (workgroup publish after the cell update)
  backward: IRC_LSTM_COOP_BWD_TAGGED=1 (tagged granules), =2 (per-wave flags)
At the C2 head shapes (B = 256, L = 64, H = 256, two directions)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

B, L, H, ND = 256, 64, 256, 2


@pytest.fixture(scope="module")
def coop_inputs(gpu):
    from irc_amd import ops

    g = torch.Generator().manual_seed(0)
    whh = (torch.randn(ND * 4 * H, H, generator=g) * 0.06).to(gpu)
    xp = (torch.randn(B * L, ND * 4 * H, generator=g) * 0.5).to(gpu)
    dy = (torch.randn(B * L, ND * H, generator=g) * 0.1).to(gpu)
    wf, wb = ops.lstm_coop_pack(whh, H, ND)
    return xp, dy, wf, wb


def _with_env(name, value, fn):
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(name)
        else:
            os.environ[name] = old


def _fwd(xp, wf):
    from irc_amd import ops

    h, g, c, hp, sync = ops.lstm_fwd_coop(xp, wf, B, L, H, ND, save=True)
    assert not ops.lstm_coop_timed_out(sync, B, ND)
    return h, g, c, hp


@pytest.mark.parametrize("env", [None, ("IRC_LSTM_COOP_SENTINELS", "1"),
                                 ("IRC_LSTM_COOP_WAVE_PUBLISH", "0")])
def test_fwd_forms_bit_identical(coop_inputs, env):
    xp, _, wf, _ = coop_inputs
    ref = _fwd(xp, wf)
    run = (lambda: _fwd(xp, wf)) if env is None else (lambda: _with_env(*env, lambda: _fwd(xp, wf)))
    for _ in range(3):
        got = run()
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


@pytest.mark.parametrize("form", ["0", "1", "2"])
def test_bwd_forms_bit_identical(coop_inputs, form):
    from irc_amd import ops

    xp, dy, wf, wb = coop_inputs
    _, g, c, _ = _fwd(xp, wf)

    def bwd():
        d, s = ops.lstm_bwd_coop(dy, wb, g, c, B, L, H, ND)
        assert not ops.lstm_coop_timed_out(s, B, ND)
        return d

    ref = bwd()
    for _ in range(3):
        assert torch.equal(_with_env("IRC_LSTM_COOP_BWD_TAGGED", form, bwd), ref)
