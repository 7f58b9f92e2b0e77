"""Restatement of the reference's multi-GPU model reduction, for the loopback harness and tests.

reduce_models follows /root/reference/coala/distributed/distributed.py:42-57 (reduce_models_only_params :60-74): all_reduce(SUM) of the sample
count, then per state_dict tensor an all_reduce(SUM) and a torch.div by the summed count (a tensor
divisor, so true division on every device), then load_state_dict. The server mixin calls the reference's
own function when COALA is importable (plugin.reduce_models).
"""
import torch.distributed as dist
import torch


def reduce_models_only_params(model, sample_sum):
    """/root/reference/coala/distributed/distributed.py:60-74: all_reduce(SUM) of the sample count, then per
    parameter an all_reduce(SUM) and param.data = torch.div(param.data, sample_sum); buffers stay as they are."""
    dist.all_reduce(sample_sum, op=dist.ReduceOp.SUM)
    if sample_sum <= 0:
        return
    for param in model.parameters():
        dist.all_reduce(param.data, op=dist.ReduceOp.SUM)
        param.data = torch.div(param.data, sample_sum)


def reduce_models(model, sample_sum):
    dist.all_reduce(sample_sum, op=dist.ReduceOp.SUM)
    if sample_sum <= 0:
        return
    state = model.state_dict()
    for k in state.keys():
        dist.all_reduce(state[k], op=dist.ReduceOp.SUM)
        state[k] = torch.div(state[k], sample_sum)
    model.load_state_dict(state)
