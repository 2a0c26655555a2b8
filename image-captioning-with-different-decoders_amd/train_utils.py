"""Gradient clipping (reference train_utils.py:2-12).

For a torch optimizer the gradients are clamped in place to [-c, c], exactly as
the reference does. For capmi.optim.Adam the clamp is fused into the
optimizer's single update kernel, so this only records the bound.
"""


def clip_gradient(optimizer, grad_clip):
    if getattr(optimizer, "fused_clamp", False):
        optimizer.set_clip(grad_clip)
        return
    for group in optimizer.param_groups:
        for param in group['params']:
            if param.grad is not None:
                param.grad.data.clamp_(-grad_clip, grad_clip)
