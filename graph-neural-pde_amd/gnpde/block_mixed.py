"""Drop-in MixedODEblock (reference src/block_mixed.py:7-63).

The Laplacian RHS integrates with a convex mix of the block-level attention and
the normalised adjacency, computed once per forward (:29-33):

    w = mean_h(attention) * (1 - sigmoid(gamma)) + edge_weight * sigmoid(gamma)

One HIP pass over the E edges (gnpde_mix_weights_f32) produces ``w`` in COO
order (``odefunc.attention_weights``, as the reference); the RHS gathers it into
CSR order once and then runs K1 like the constant block ('mixed' weight source,
function_laplacian_diffusion.py:50-53).  Gradients reach gamma, the attention
(and through it Q, K and x) and the edge weights: ``_MixWeights`` carries the
RHS's SDDMM weight gradient back through the mix.
"""
import torch
from torch import nn

from . import ops
from .base_classes import ODEblock
from .function_transformer_attention import SpGraphTransAttentionLayer
from .integrator import odeint, odeint_adjoint


class _MixWeights(torch.autograd.Function):
    """w = mean_h(att) (1 - s) + ew s, s = sigmoid(gamma) (src/block_mixed.py:29-33)."""

    @staticmethod
    def forward(ctx, att, edge_weight, gamma):
        ctx.save_for_backward(att, edge_weight, gamma)
        return ops.mix_weights(att.detach(), edge_weight.detach(), gamma.detach())

    @staticmethod
    def backward(ctx, gw):
        att, ew, gamma = ctx.saved_tensors
        s = torch.sigmoid(gamma.detach().float())
        g_att = g_ew = g_gamma = None
        if ctx.needs_input_grad[0]:
            H = att.shape[2] if att.dim() == 3 else 1
            g = gw * (1 - s)
            g_att = (g / H).unsqueeze(-1).expand_as(att).contiguous() if att.dim() == 3 else g
        if ctx.needs_input_grad[1]:
            g_ew = gw * s
        if ctx.needs_input_grad[2]:
            mean = ops.mix_weights(att.detach())
            d = (gw.double() * (ew.detach().double() - mean.double())).sum()
            g_gamma = (d * (s * (1 - s)).double()).reshape(gamma.shape).to(gamma.dtype)
        return g_att, g_ew, g_gamma


class MixedODEblock(ODEblock):
    def __init__(self, odefunc, regularization_fns, opt, device, t=torch.tensor([0, 1]), gamma=0.):
        super(MixedODEblock, self).__init__(odefunc, regularization_fns, opt, device, t)
        self.device = device
        self.odefunc = self._new_odefunc(odefunc, opt, device)  # the integrated copy (src/block_mixed.py:12)
        self.train_integrator = odeint_adjoint if opt.get('adjoint', False) else odeint
        self.test_integrator = odeint
        self.set_tol()
        # parameter trading off between attention and the Laplacian (:20)
        self.gamma = nn.Parameter(gamma * torch.ones(1))
        self.multihead_att_layer = SpGraphTransAttentionLayer(opt['hidden_dim'], opt['hidden_dim'], opt, device)
        if device is not None:
            self.multihead_att_layer = self.multihead_att_layer.to(device)

    def get_attention_weights(self, x):
        attention, values = self.multihead_att_layer(x, self.odefunc.edge_index)
        return attention

    def get_mixed_attention(self, x):
        """(1 - sigmoid(gamma)) * mean_h(attention) + sigmoid(gamma) * edge_weight (:29-33), [B,E] COO order."""
        attention = self.get_attention_weights(x)
        return _MixWeights.apply(attention, self.odefunc.edge_weight, self.gamma)

    def forward(self, x, graph_data, y=None):
        self.reset_graph_data(graph_data, x.dtype, y)
        self.odefunc.attention_weights = self.get_mixed_attention(x)
        return self._integrate(x, {'step_size': self.opt.get('step_size')})

    def __repr__(self):
        return self.__class__.__name__ + '( Time Interval ' + str(self.t[0].item()) + ' -> ' + \
            str(self.t[1].item()) + ")"
