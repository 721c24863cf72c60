"""CPU tests of the in-place paths (no kernels run): HF.CatSlot, the decoder concatenation buffer
whose tail the skip's producer writes in place (functional.py CatSlot; MixConvNeXtML.py:229-236
upSample cat) -- its aliasing and the holds() check that decides whether a concat node may skip the
copy, where a false positive would let a node overwrite a live tensor's head; pw_mlp's acc
validation; and the nested gradient-box merge rule (functional._acc_target).
"""
import torch

from dsgan_hip import functional as HF


def _slot(N=2, Ch=3, Ct=5, H=4, W=4):
    return HF.CatSlot(N, Ch, Ct, H, W, torch.empty(1))


def test_tail_and_whole_alias_the_buffer():
    s = _slot()
    t, w = s.tail(), s.whole()
    assert t.shape == (2, 5, 4, 4) and w.shape == (2, 8, 4, 4)
    assert t._base is None and w._base is None   # aliases, not autograd views of the buffer
    t.fill_(1.0)
    w[:, :3].fill_(2.0)
    assert torch.equal(s.buf[:, 3:], torch.ones(2, 5, 4, 4))
    assert torch.equal(s.buf[:, :3], torch.full((2, 3, 4, 4), 2.0))
    assert torch.equal(w, s.buf)
    assert t.stride() == s.buf.stride()


def test_holds_its_own_tail_and_views_of_it():
    s = _slot()
    t = s.tail()
    assert s.holds(t, 3)
    assert s.holds(t.view_as(t), 3)   # HF.share returns a view_as alias


def test_holds_refuses_everything_else():
    s = _slot()
    t = s.tail()
    assert not s.holds(t, 4)                          # another head width
    assert not s.holds(t.clone(), 3)                  # same values, other storage
    assert not s.holds(s.buf[:, :5], 3)               # the head region
    assert not s.holds(_slot().tail(), 3)             # another slot's tail
    assert not s.holds(t[:, :4], 3)                   # fewer channels
    assert not s.holds(t.contiguous().view(2, 5, 4, 4).clone(), 3)
    assert not s.holds(None, 3)
    other = torch.empty(2, 8, 4, 4)
    assert not s.holds(other[:, 3:], 3)               # same geometry in a foreign buffer


def test_pw_mlp_refuses_a_bad_acc_before_any_launch():
    """pw_mlp(acc=) sums the block into acc in place: anything but a dense fp32 [N,P,H,W] tensor,
    or acc together with a slot, is refused before a kernel is issued."""
    import pytest
    N, C, P, H = 2, 4, 8, 4
    h, x = torch.zeros(N, C, H, H), torch.zeros(N, C, H, H)
    prm = [torch.zeros(4 * C, C), torch.zeros(4 * C), torch.zeros(P, 4 * C), torch.zeros(P), torch.zeros(P, C, 1, 1)]
    for bad in (torch.zeros(N, P + 1, H, H), torch.zeros(N, P, H, H, dtype=torch.float64),
                torch.zeros(N, P, H, 2 * H)[..., ::2]):
        with pytest.raises(ValueError, match="acc"):
            HF.pw_mlp(h, x, *prm, acc=bad)
    with pytest.raises(ValueError, match="acc"):
        HF.pw_mlp(h, x, *prm, slot=HF.CatSlot(N, P, P, H, H, h), acc=torch.zeros(N, P, H, H))


def test_nested_grad_box_merges_only_into_an_owned_outer_buffer():
    """_acc_target on a box nested in another (share of a shared tensor): it merges into the outer
    box's buffer only when that buffer is owned (freshly computed, safe to accumulate into), never
    into a borrowed one (a grad autograd handed over), and an inner box with a buffer of its own
    keeps it."""
    outer, inner = HF._GradBox(), HF._GradBox()
    inner.outer = outer
    assert HF._acc_target(inner) == (None, False)             # outer empty: nothing to merge into
    g = torch.zeros(2, 3)
    outer.buf, outer.owned = g, False
    assert HF._acc_target(inner) == (None, False) and not inner.merged   # borrowed: no merge
    outer.owned = True
    buf, acc = HF._acc_target(inner)
    assert buf is g and acc and inner.merged and inner.owned
    own = HF._GradBox()
    own.outer, own.buf, own.owned = outer, torch.ones(2, 3), True
    buf, acc = HF._acc_target(own)
    assert buf is own.buf and buf is not g and not own.merged
