"""Drop-in HardAttODEblock (reference src/block_transformer_hard_attention.py:6-99).

Eval (:58-60): the RHS integrates over the full graph with the head-mean of
the block-level attention — one HIP pass (gnpde_mix_weights_f32) then K1.

Training (:42-57): edges whose mean attention exceeds the (1 - att_samp_pct)
quantile are kept and their weights renormalised per softmax group (:32-35);
the RHS then integrates over the sampled graph.  The threshold is a device
radix sort + torch.quantile's interpolation (gnpde_quantile_f32), the
renormalisation a fixed-order per-group pass (gnpde_group_normalize_f32).  With
the Laplacian RHS (which reads ``attention_weights``) the dropped edges keep weight
0 on the full graph (gnpde_threshold_mask_f32) and K1 gathers the retained edges
only, compacted inside the full plan's items on the device (gnpde_compact_items_f32,
ops.CompactWeights): no graph rebuilt per forward, no host read.  The transformer /
GAT RHS recomputes its attention over ``odefunc.edge_index`` at every evaluation
(src/function_transformer_attention.py:49), so there the edge list itself is
compacted (:54), as in the reference.  The sampling runs under no_grad exactly as
in the reference, so training differentiates the RHS through x, alpha_train and
beta_train only — which the Laplacian backward provides.

The fork's training branch cannot run as written (SURVEY.md §0.5 family): it
indexes the batched [B,2,E] edge list with ``mask.T`` (:54) and takes
``edge_index[attention_norm_idx]`` along the batch axis (:33).  This module
follows the upstream single-graph semantics (B = 1; ``index`` = source row
for attention_norm_idx 0, destination row for 1); parity for that branch is
against the oracle only.  ``use_flux`` broadcasts [B,1,E] against [1,1,C]
(:46-50) and is broken for E != C: it raises.
"""
import torch

from . import ops
from .base_classes import ODEblock
from .function_transformer_attention import SpGraphTransAttentionLayer
from .integrator import odeint, odeint_adjoint


class HardAttODEblock(ODEblock):
    def __init__(self, odefunc, regularization_fns, opt, device, t=torch.tensor([0, 1]), gamma=0.5):
        super(HardAttODEblock, self).__init__(odefunc, regularization_fns, opt, device, t)
        self.device = device
        # the integrated copy (src/block_transformer_hard_attention.py:11)
        self.odefunc = self._new_odefunc(odefunc, opt, device)
        assert opt['att_samp_pct'] > 0 and opt['att_samp_pct'] <= 1, "attention sampling threshold must be in (0,1]"
        self.train_integrator = odeint_adjoint if opt.get('adjoint', False) else odeint
        self.test_integrator = odeint
        self.set_tol()
        if opt['function'] not in {'GAT', 'transformer'}:
            self.multihead_att_layer = SpGraphTransAttentionLayer(opt['hidden_dim'], opt['hidden_dim'], opt, device,
                                                                  edge_weights=self.odefunc.edge_weight)
            if device is not None:
                self.multihead_att_layer = self.multihead_att_layer.to(device)

    def get_attention_weights(self, x):
        if self.opt['function'] not in {'GAT', 'transformer'}:
            attention, values = self.multihead_att_layer(x, self.data_edge_index)
        else:
            attention, values = self.odefunc.multihead_att_layer(x, self.data_edge_index)
        return attention

    def renormalise_attention(self, attention):
        """attention [B,E'] over odefunc.edge_index / (its group sum + 1e-16) (:32-35)."""
        g = self.odefunc.graph_for(int(self.num_nodes))
        grouped = g.csr if int(self.opt['attention_norm_idx']) == 0 else g.csc
        return ops.group_normalize(grouped, attention.reshape(-1)).reshape(attention.shape)

    def sample_edges(self, x):
        """Training-mode attention sampling (:42-57): (edge_index [1,2,E], weights [1,E]).

        The retained edges are those whose mean attention exceeds the
        (1 - att_samp_pct) quantile; the module keeps the FULL edge list and gives
        the dropped edges weight 0 (gnpde_threshold_mask_f32), renormalising per
        softmax group over the full graph.  Zero weights add exact zeros to every
        row and group sum, so the integrated RHS is the RHS over the compacted edge
        list of the reference (:54-56) — while the CSR, the work plans and the
        node numbering built once per graph serve every training forward (no
        per-forward graph rebuild, no host-syncing boolean index; one host read
        for the reference's 'retaining' line)."""
        if self.opt.get('use_flux', False):
            raise NotImplementedError("gnpde: use_flux is broken in the reference (broadcasts [B,1,E] against "
                                      "[1,1,C], block_transformer_hard_attention.py:46-50)")
        ei = self.data_edge_index
        if ei.shape[0] != 1:
            raise NotImplementedError("gnpde: hard-attention sampling keeps a different edge count per graph; "
                                      "the reference's batched branch is broken (:54) and only B = 1 is supported")
        with torch.no_grad():
            mean_att = ops.mix_weights(self.get_attention_weights(x))
            threshold = ops.quantile(mean_att, 1 - self.opt['att_samp_pct'])
            if self.reads_weights():
                masked, kept = ops.threshold_mask(mean_att, threshold)
                self.odefunc.edge_index = ei
                weights = self.renormalise_attention(masked)
            else:
                # the transformer / GAT RHS attends over odefunc.edge_index itself: the compacted list (:54)
                mask = (mean_att > threshold).reshape(-1)
                ei = ei[:, :, mask]
                kept = ei.shape[2]
                self.odefunc.edge_index = ei
                weights = self.renormalise_attention(mean_att.reshape(1, -1)[:, mask])
        self.retained = kept
        print('retaining {} of {} edges'.format(int(kept), self.data_edge_index.shape[2]))
        return ei, weights

    def reads_weights(self):
        """Whether the integrated RHS reads ``attention_weights`` (the Laplacian) rather than
        recomputing its attention over ``edge_index`` (ODEFuncTransformerAtt / GAT)."""
        return hasattr(self.odefunc, '_weights_tensor')

    def forward(self, x, graph_data, y=None):
        self.reset_graph_data(graph_data, x.dtype, y)
        # the sampled graph's zero weights: K1 over the retained edges only (ops.CompactWeights)
        for f in (self.odefunc, self.reg_odefunc.odefunc):
            f.compact_sampled = bool(self.training) and self.reads_weights()
        if self.training:
            edge_index, weights = self.sample_edges(x)
            self.odefunc.edge_index = edge_index
            self.odefunc.attention_weights = weights
        else:
            self.odefunc.edge_index = self.data_edge_index
            att = self.get_attention_weights(x)
            # head mean (:60); with autograd recording the torch mean keeps the attention's graph
            self.odefunc.attention_weights = att.mean(dim=2) if att.requires_grad else ops.mix_weights(att)
        self.reg_odefunc.odefunc.edge_index = self.odefunc.edge_index
        self.reg_odefunc.odefunc.edge_weight = self.odefunc.edge_weight
        self.reg_odefunc.odefunc.attention_weights = self.odefunc.attention_weights
        return self._integrate(x, {'step_size': self.opt.get('step_size')})

    def __repr__(self):
        return self.__class__.__name__ + '( Time Interval ' + str(self.t[0].item()) + ' -> ' + \
            str(self.t[1].item()) + ")"
