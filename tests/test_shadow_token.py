"""FlatParamSpace.mark_shadow_fresh: an optimizer step that wrote the bf16 shadow lets the next
refresh_shadow skip its cast -- unless the weights changed since (autograd version counters of the
parameters or the flat buffer, or a non-autograd writer: note_param_write)."""
import torch

from kungfu_amd.parallel.flat import FlatParamSpace, axpby_, note_param_write


def _space():
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.Linear(4, 2))
    sp = FlatParamSpace(list(m.parameters()))
    sp.enable_shadow()
    return m, sp


def _stale(sp):
    return not torch.equal(sp.flat_shadow, sp.flat_param.to(torch.bfloat16))


def test_fresh_shadow_skips_the_cast_once():
    m, sp = _space()
    with torch.no_grad():
        sp.flat_param.data.add_(1.0)  # a writer the token cannot see, standing in for the step kernel
    sp.flat_shadow.copy_(sp.flat_param)  # ... which also wrote the shadow
    sp.mark_shadow_fresh()
    gen = sp.shadow_gen
    sp.flat_shadow.zero_()  # marker: a skipped refresh leaves it
    sp.refresh_shadow()
    assert sp.shadow_gen == gen + 1 and sp.flat_shadow.abs().sum() == 0
    sp.refresh_shadow()  # the token is consumed: the next refresh casts
    assert not _stale(sp)


def test_param_edits_invalidate_the_token():
    m, sp = _space()
    for edit in (lambda: m[0].weight.mul_(2.0), lambda: sp.flat_param.add_(0.5),
                 lambda: axpby_(sp.flat_param, sp.flat_param.clone(), 0.5, 0.5), note_param_write):
        sp.mark_shadow_fresh()
        with torch.no_grad():
            edit()
        sp.refresh_shadow()
        assert not _stale(sp)
