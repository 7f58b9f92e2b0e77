"""FedAvg over decoded modules — restatement of /root/reference/coala/server/strategies.py.

federated_averaging: strategies.py:6-29 — weighted sum of EVERY state_dict entry (fp32 and int64
buffers alike), then torch.div by the total weight (int64 entries become float, as in the reference).
weighted_sum: strategies.py:57-90 — params *= w0, then += model_i[name] * w_i in client order.
*_only_params: strategies.py:32-54, 93-124 — the same over named_parameters() only; the result keeps
models[0]'s buffers (deepcopy(models[0])), and the average divides with `params / total`.
"""
import copy

import torch


def weighted_sum(models, weights):
    if not models or not weights:
        return None, 0
    total = sum(weights)
    if total == 0:
        weights = [1 for _ in models]
    model = copy.deepcopy(models[0])
    acc = copy.deepcopy(models[0].state_dict())
    states = [dict(m.state_dict()) for m in models]
    with torch.no_grad():
        for name, params in acc.items():
            params *= weights[0]
            for i in range(1, len(models)):
                params += states[i][name] * weights[i]
            acc[name] = params
    model.load_state_dict(acc)
    return model, total


def federated_averaging(models, weights):
    if not models:
        return None
    if not weights or sum(weights) == 0:
        weights = [1 for _ in models]
    model, total = weighted_sum(models, weights)
    state = model.state_dict()
    with torch.no_grad():
        for name, params in state.items():
            state[name] = torch.div(params, total)
    model.load_state_dict(state)
    return model


def weighted_sum_only_params(models, weights):
    if not models or not weights:
        return None, 0
    total = sum(weights)
    if total == 0:
        weights = [1 for _ in models]
    model = copy.deepcopy(models[0])
    acc = dict(model.named_parameters())
    others = [dict(m.named_parameters()) for m in models]
    with torch.no_grad():
        for name, params in acc.items():
            params *= weights[0]
            for i in range(1, len(models)):
                params += others[i][name] * weights[i]
            acc[name].set_(params)
    return model, total


def federated_averaging_only_params(models, weights):
    if not models:
        return None
    if not weights or sum(weights) == 0:
        weights = [1 for _ in models]
    model, total = weighted_sum_only_params(models, weights)
    params = dict(model.named_parameters())
    with torch.no_grad():
        for name in params:
            params[name].set_(params[name] / total)
    return model
