"""Drop-in ODEFunc / ODEblock base classes (reference src/base_classes.py).

Same constructor signatures, attribute contract and state_dict keys as the
reference, so ``GNN.__init__`` (src/GNN.py:12-15) and the torchdiffeq-style
loop use them unchanged:

* ``ODEFunc(opt, device)`` — src/base_classes.py:116-134: attributes
  ``edge_index``, ``edge_weight``, ``attention_weights``, ``x0``, ``nfe``,
  parameters ``alpha_train``, ``beta_train`` (0-d, init 0), ``alpha_sc``,
  ``beta_sc``.  Adds a per-graph CSR cache: the first RHS call after
  ``edge_index`` changes builds the device CSR + plan once; every later call
  reuses it.
* ``ODEblock(odefunc, regularization_fns, opt, device, t)`` —
  src/base_classes.py:33-98: ``odefunc``, ``reg_odefunc.odefunc``,
  ``train_integrator``/``test_integrator``, ``set_x0``, ``set_tol``,
  ``reset_tol``, ``reset_graph_data``, ``set_time``.  Module layout as the
  reference: ``ODEblock.__init__`` builds an ODEFunc and wraps it in
  ``reg_odefunc`` (:40, :43); every concrete block then builds a SECOND
  ODEFunc as ``self.odefunc`` (src/block_constant.py:11,
  src/block_transformer_attention.py:11, src/block_mixed.py:12,
  src/block_transformer_hard_attention.py:11), which is the one the solver
  integrates.  A reference ``state_dict`` therefore holds both
  ``odefunc.*`` and ``reg_odefunc.odefunc.*`` and loads here unchanged, and
  ``GNN.getNFE`` (src/base_classes.py:174-176) sums the two counters.
* ``GraphData`` — src/base_classes.py:100-113.
"""
import os

import torch
from torch import nn

from . import ops
from ._cache import _tensor_key  # noqa: F401  (re-exported for the function modules)
from .integrator import odeint, odeint_adjoint
from .utils import get_rw_adj, gcn_norm_fill_val


# GNPDE_COMPACT_SAMPLED=0: the sampled hard-attention graph stays the masked full graph
COMPACT_SAMPLED = os.environ.get('GNPDE_COMPACT_SAMPLED', '1') != '0'


class GraphData(object):
    def __init__(self):
        super(GraphData, self).__init__()
        self.edge_index = None
        self.edge_attr = None
        self.num_nodes = None

    def new_graph(self, edge_index, num_nodes, edge_attr=None):
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.num_nodes = num_nodes

    def __repr__(self):
        return self.__class__.__name__




class ODEFunc(nn.Module):
    """Base RHS module (src/base_classes.py:116-134)."""

    # f(t, x) does not read t (every RHS of the path: src/function_laplacian_diffusion.py:60-77,
    # src/function_transformer_attention.py:44-59): the integrator may replay captured steps whose
    # recorded stage times are stale, and evaluate the initial-step probe without reading h0 back
    autonomous = True

    def __init__(self, opt, device):
        super(ODEFunc, self).__init__()
        self.opt = opt
        self.device = device
        self.edge_index = None
        self.edge_weight = None
        self.attention_weights = None
        self.alpha_train = nn.Parameter(torch.tensor(0.0))
        self.beta_train = nn.Parameter(torch.tensor(0.0))
        self.x0 = None
        self.nfe = 0
        self.alpha_sc = nn.Parameter(torch.ones(1))
        self.beta_sc = nn.Parameter(torch.ones(1))
        self._graph = None
        self._graph_key = None
        self._w_cache = {}
        self._layout = None  # the NodeLayout a fixed-grid solve runs in (gnpde.integrator), else None
        # weights with zeros on dropped edges (HardAttODEblock training's sampled graph): csr_weights
        # hands K1 the retained edges compacted inside the plan's items (ops.CompactWeights)
        self.compact_sampled = False

    def graph_for(self, x):
        """Device CSR of ``self.edge_index`` for node count x.shape[1] (or x, an
        int node count) — cached per edge_index tensor version."""
        if self.edge_index is None:
            raise RuntimeError("%s: edge_index is not set (the ODE block sets it in reset_graph_data)" %
                               self.__class__.__name__)
        n = x if isinstance(x, int) else int(x.shape[1])
        key = (_tensor_key(self.edge_index), n)
        if self._graph is None or key != self._graph_key:
            chunk = self.opt.get('gnpde_chunk') if isinstance(self.opt, dict) else None  # None: ops.auto_chunk
            self._graph = ops.GraphCSR(self.edge_index, n, chunk=chunk)
            self._graph_key = key
            self._w_cache = {}
        if self._layout is not None:
            return self._layout.graph
        return self._graph

    def supports_node_layout(self):
        """True when every operand of the RHS is per node or per edge in COO order,
        so the integrator may run it on a renumbered state (ops.NodeLayout)."""
        return False

    def node_layout(self, x):
        """The locality numbering the fixed-grid integrator keeps this solve's
        state in (ops.NodeLayout, built once per graph), or None: not supported,
        a layout already active, or a state too small to gain from it."""
        if self._layout is not None or not self.supports_node_layout() or x.dim() != 3:
            return None
        if not ops.layout_worthwhile(x.shape[0] * x.shape[1], x.shape[-1], x.element_size()):
            return None
        return self.graph_for(x).node_layout

    def csr_weights(self, g, w, tag, transpose=False):
        """COO-order weights (or [B,E,h] attention -> head mean) in CSR (or CSC) order,
        cached per source tensor (identity and version).

        Under no_grad a changed source (the attention blocks hand over a new
        ``attention_weights`` tensor every forward) is gathered IN PLACE into the
        buffer of the previous one when that buffer was made under no_grad and
        never given to autograd: the integrator's captured step graphs read that
        buffer, so they keep replaying with the new weights instead of being
        re-captured every forward.  Buffers an autograd call has seen are never
        overwritten (its backward may still read them)."""
        compact = bool(self.compact_sampled) and COMPACT_SAMPLED
        tag = (tag, transpose, compact)
        key = (tag, _tensor_key(w), id(g))
        hit = self._w_cache.get(tag)
        grad = torch.is_grad_enabled()
        if hit is not None and hit[0] == key:
            if grad and hit[2]:
                self._w_cache[tag] = (hit[0], hit[1], False)
            return hit[1]
        src = w.detach().float() if w.dtype != torch.float32 else w.detach()
        reuse = hit is not None and hit[2] and not grad and hit[0][2] == id(g)
        prev = hit[1] if reuse else None
        if compact:
            # the sampled graph (HardAttODEblock training): the retained edges compacted inside the
            # plan's items on the device (ops.CompactWeights), refreshed in place like the weights
            full = g.gather_weights(src, transpose=transpose, out=prev.full if prev is not None else None)
            wc = ops.compact_weights(g.csc if transpose else g.csr, full, transpose, out=prev)
        else:
            wc = g.gather_weights(src, transpose=transpose, out=prev)
        self._w_cache[tag] = (key, wc, not grad)
        return wc

    def stable_x0(self, x):
        """x0 in x's dtype and (zero-padded) width, in a buffer that stays the same
        across set_x0 calls of the same shape (refreshed in place): what the fused
        Runge-Kutta stages and their captured step graphs read.  ODEblock.set_x0
        clones x0 every forward (src/base_classes.py:53-55), so reading self.x0
        directly would pin a captured graph to a stale pointer."""
        x0 = self.x0
        if x0 is None:
            raise RuntimeError("%s: add_source needs x0 (ODEblock.set_x0)" % self.__class__.__name__)
        lay = self._layout
        key = (_tensor_key(x0), id(lay) if lay is not None else None)
        slot = '_x0_buf' if lay is None else '_x0_buf_layout'  # one stable buffer per numbering
        shape = tuple(x0.shape[:-1]) + (x.shape[-1],)
        hit = getattr(self, slot, None)
        if hit is not None and hit[0] == key and hit[1].shape == shape and hit[1].dtype == x.dtype and \
                hit[1].device == x.device:
            return hit[1]
        if hit is not None and hit[1].shape == shape and hit[1].dtype == x.dtype and hit[1].device == x.device:
            buf = hit[1]
        else:
            buf = torch.zeros(shape, dtype=x.dtype, device=x.device)
        src = x0.detach()
        buf[..., :x0.shape[-1]].copy_(src if lay is None else lay.to_internal(src))
        setattr(self, slot, (key, buf))
        return buf

    def __repr__(self):
        return self.__class__.__name__


class RegularizedODEfunc(nn.Module):
    """Holder with the reference's ``reg_odefunc.odefunc`` attribute path
    (src/regularized_ODE_function.py).  The kinetic-energy / Jacobian
    regularisers are OUT OF SCOPE (off by default, broken in the fork)."""

    def __init__(self, odefunc, regularization_fns):
        super(RegularizedODEfunc, self).__init__()
        self.odefunc = odefunc
        self.regularization_fns = regularization_fns

    def forward(self, t, state):
        raise NotImplementedError("gnpde: ODE regularisation terms are out of scope (SURVEY.md §2 row 12)")


class ODEblock(nn.Module):
    """src/base_classes.py:33-98."""

    def __init__(self, odefunc, regularization_fns, opt, device, t):
        super(ODEblock, self).__init__()
        self.opt = opt
        self.t = t
        self.device = device
        self.aug_dim = 2 if opt.get('augment', False) else 1
        self.odefunc = odefunc(self.aug_dim * opt['hidden_dim'], self.aug_dim * opt['hidden_dim'], opt, device)
        self.nreg = len(regularization_fns)
        self.reg_odefunc = RegularizedODEfunc(self.odefunc, regularization_fns)
        self.train_integrator = odeint_adjoint if opt.get('adjoint', False) else odeint
        self.test_integrator = None
        self.set_tol()
        self._prep_key = None
        self._prep = None

    def _new_odefunc(self, odefunc, opt, device):
        """The block's own ODEFunc, built after ODEblock.__init__ exactly as the
        reference blocks do (e.g. src/block_constant.py:10-11); ``reg_odefunc``
        keeps the first copy."""
        self.aug_dim = 2 if opt.get('augment', False) else 1
        return odefunc(self.aug_dim * opt['hidden_dim'], self.aug_dim * opt['hidden_dim'], opt, device)

    def set_x0(self, x0):
        self.odefunc.x0 = x0.clone().detach()
        self.reg_odefunc.odefunc.x0 = x0.clone().detach()

    def set_tol(self):
        self.atol = self.opt.get('tol_scale', 1) * 1e-7
        self.rtol = self.opt.get('tol_scale', 1) * 1e-9
        if self.opt.get('adjoint', False):
            self.atol_adjoint = self.opt.get('tol_scale_adjoint', 1) * 1e-7
            self.rtol_adjoint = self.opt.get('tol_scale_adjoint', 1) * 1e-9

    def reset_tol(self):
        self.atol = 1e-7
        self.rtol = 1e-9
        self.atol_adjoint = 1e-7
        self.rtol_adjoint = 1e-9

    def reset_graph_data(self, data, dtype, y=None):
        """src/base_classes.py:70-90 with the intended normalisation semantics
        (gnpde.utils): self-loops (weight self_loop_weight) + rw (norm_dim=1) or
        symmetric gcn normalisation.  The reference's second
        add_remaining_self_loops (:83-85) is a no-op once every node has a
        loop and is skipped.  Cached on (edge_index, edge_attr) identity, so a
        model that passes the same graph every forward prepares it once.

        The weights are built in fp32 whatever the state dtype: the reference
        passes ``dtype=x.dtype`` (:77, :82), which under a bf16 state would form
        degree sums in bf16 (integers exact only to 256) and round every weight
        to 8 bits before the fp32 aggregation reads it."""
        if data is not None:
            dtype = torch.float32
            key = (_tensor_key(data.edge_index), _tensor_key(data.edge_attr), int(data.num_nodes),
                   self.opt.get('data_norm', 'rw'), float(self.opt.get('self_loop_weight', 0)))
            if key != self._prep_key:
                self.num_nodes = data.num_nodes
                ea = data.edge_attr.float() if data.edge_attr is not None else None
                if self.opt.get('data_norm', 'rw') == 'rw':
                    edge_index, edge_weight = get_rw_adj(data.edge_index, edge_weight=ea, norm_dim=1,
                                                         fill_value=self.opt['self_loop_weight'],
                                                         num_nodes=data.num_nodes, dtype=dtype)
                else:
                    edge_index, edge_weight = gcn_norm_fill_val(data.edge_index, edge_weight=ea,
                                                                fill_value=self.opt['self_loop_weight'],
                                                                num_nodes=data.num_nodes, dtype=dtype)
                dev = self.device if self.device is not None else edge_index.device
                self._prep = (edge_index.to(dev), edge_weight.to(dev))
                self._prep_key = key
            edge_index, edge_weight = self._prep
            self.data_edge_index = edge_index
            self.odefunc.edge_index = edge_index
            self.odefunc.edge_weight = edge_weight
            self.reg_odefunc.odefunc.edge_index = edge_index
            self.reg_odefunc.odefunc.edge_weight = edge_weight
        self.odefunc.y = y

    def set_time(self, time):
        self.t = torch.tensor([0, time]).to(self.device)

    def _integrate(self, x, options):
        if self.training and self.nreg > 0:
            raise NotImplementedError("gnpde: ODE regularisation terms are out of scope (SURVEY.md §2 row 12)")
        integrator = self.train_integrator if self.training else self.test_integrator
        t = self.t.type_as(x)
        if self.opt.get('adjoint', False) and self.training:
            # block_constant.py:34-44: adjoint method / step size / tolerances of their own
            a_opts = {'step_size': self.opt.get('adjoint_step_size', options.get('step_size'))}
            if 'max_iters' in options:
                a_opts['max_iters'] = options['max_iters']
            state_dt = integrator(self.odefunc, x, t, method=self.opt['method'], options=options,
                                  adjoint_method=self.opt.get('adjoint_method', self.opt['method']),
                                  adjoint_options=a_opts, atol=self.atol, rtol=self.rtol,
                                  adjoint_atol=self.atol_adjoint, adjoint_rtol=self.rtol_adjoint)
        else:
            state_dt = integrator(self.odefunc, x, t, method=self.opt['method'], options=options, atol=self.atol,
                                  rtol=self.rtol)
        return state_dt[1]

    def __repr__(self):
        return self.__class__.__name__ + '( Time Interval ' + str(self.t[0].item()) + ' -> ' + \
            str(self.t[1].item()) + ")"
