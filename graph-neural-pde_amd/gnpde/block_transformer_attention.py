"""Drop-in AttODEblock (reference src/block_transformer_attention.py:6-69).

The block-level SpGraphTransAttentionLayer computes the multi-head attention
once per forward (:31); the Laplacian RHS then integrates with its head-mean
(function_laplacian_diffusion.py:45-49), gathered once into CSR order.
"""
import torch

from .base_classes import ODEblock
from .function_transformer_attention import SpGraphTransAttentionLayer
from .integrator import odeint, odeint_adjoint


class AttODEblock(ODEblock):
    def __init__(self, odefunc, regularization_fns, opt, device, t=torch.tensor([0, 1]), gamma=0.5):
        super(AttODEblock, self).__init__(odefunc, regularization_fns, opt, device, t)
        self.device = device
        # the integrated copy (src/block_transformer_attention.py:11)
        self.odefunc = self._new_odefunc(odefunc, opt, device)
        self.train_integrator = odeint_adjoint if opt.get('adjoint', False) else odeint
        self.test_integrator = odeint
        self.set_tol()
        self.multihead_att_layer = SpGraphTransAttentionLayer(opt['hidden_dim'], opt['hidden_dim'], opt, device,
                                                              edge_weights=self.odefunc.edge_weight)
        if device is not None:
            self.multihead_att_layer = self.multihead_att_layer.to(device)

    def get_attention_weights(self, x):
        attention, values = self.multihead_att_layer(x, self.odefunc.edge_index)
        return attention

    def forward(self, x, graph_data, y=None):
        self.reset_graph_data(graph_data, x.dtype, y)
        self.odefunc.attention_weights = self.get_attention_weights(x)
        self.reg_odefunc.odefunc.attention_weights = self.odefunc.attention_weights
        return self._integrate(x, {'step_size': self.opt.get('step_size')})

    def __repr__(self):
        return self.__class__.__name__ + '( Time Interval ' + str(self.t[0].item()) + ' -> ' + \
            str(self.t[1].item()) + ")"
