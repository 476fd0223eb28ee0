"""Drop-in LaplacianODEFunc (reference src/function_laplacian_diffusion.py:15-77).

``forward(t, x)`` computes ``f = sigma(alpha_train) * (A x - x) [+ beta_train * x0]``
with one HIP launch (K1, gnpde_spmm_rhs_f32): CSR gather-aggregate with the
epilogue fused.  The weight source follows ``opt['block']`` exactly as the
reference (:45-57): 'attention' -> head-mean of ``attention_weights [B,E,h]``,
'mixed'/'hard_attention' -> ``attention_weights [B,E]``, otherwise
``edge_weight [B,E]``.  Duplicated edges are summed, as the reference's
COO -> to_dense does.

Gradients: x (the same K1 over the CSC for A^T),
alpha_train / beta_train (two reductions) and the edge weights — whichever
tensor the block handed over (edge_weight [B,E], or attention_weights [B,E] /
[B,E,h] whose head mean is taken): an SDDMM g_w[e] = a <gf[src], x[dst]>
(gnpde_sddmm_f32) written straight into the COO layout of that tensor, so
autograd carries it on into the attention that produced it.
"""
import torch
from torch import nn

from . import ops
from .base_classes import ODEFunc
from .utils import MaxNFEException


class _LaplacianRHS(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, alpha_train, beta_train, w_src, g, w_csr, w_csc_fn, x0, alpha_sigmoid, add_source):
        f = ops.spmm_rhs(g, w_csr, x, x0=x0, alpha=alpha_train.detach(), beta=beta_train.detach(), rhs=True,
                         alpha_sigmoid=alpha_sigmoid, add_source=add_source)
        ctx.save_for_backward(x, alpha_train, beta_train)
        ctx.g, ctx.w_csr, ctx.w_csc_fn, ctx.x0 = g, w_csr, w_csc_fn, x0
        ctx.alpha_sigmoid, ctx.add_source = alpha_sigmoid, add_source
        ctx.w_heads = w_src.shape[2] if w_src.dim() == 3 else 1
        ctx.w_shape = w_src.shape
        return f

    @staticmethod
    def backward(ctx, gf):
        x, alpha_train, beta_train = ctx.saved_tensors
        gf = gf.contiguous()
        g = ctx.g
        gx = ga = gb = None
        if ctx.needs_input_grad[0]:
            # d/dx [a (A x - x)] applied to gf = a (A^T gf - gf): K1 over the CSC
            gx = ops.spmm_rhs(g, ctx.w_csc_fn(), gf, alpha=alpha_train.detach(), rhs=True,
                              alpha_sigmoid=ctx.alpha_sigmoid, transpose=True)
        if ctx.needs_input_grad[1]:
            one = torch.ones((), dtype=torch.float32, device=x.device)
            d = ops.spmm_rhs(g, ctx.w_csr, x.detach(), alpha=one, rhs=True, alpha_sigmoid=False)  # A x - x
            s = ops.dot(gf, d).to(alpha_train.dtype)  # fp64 accumulation, fixed order
            if ctx.alpha_sigmoid:
                sg = torch.sigmoid(alpha_train.detach())
                s = s * sg * (1 - sg)
            ga = s.reshape(alpha_train.shape)
        if ctx.needs_input_grad[2]:
            if ctx.add_source:
                gb = ops.dot(gf, ctx.x0.float()).to(beta_train.dtype).reshape(beta_train.shape)
            else:
                gb = torch.zeros_like(beta_train)
        gw = None
        if ctx.needs_input_grad[3]:
            # d f[src] / d w_e = a x[dst]  ->  g_w[e] = a <gf[src], x[dst]> (/ heads for a head mean)
            gw = ops.sddmm(g, gf, x.detach(), heads=ctx.w_heads, alpha=alpha_train.detach(),
                           alpha_sigmoid=ctx.alpha_sigmoid).view(ctx.w_shape)
        return gx, ga, gb, gw, None, None, None, None, None, None


class LaplacianODEFunc(ODEFunc):

    # currently requires in_features = out_features (as the reference)
    def __init__(self, in_features, out_features, opt, device):
        super(LaplacianODEFunc, self).__init__(opt, device)
        self.in_features = in_features
        self.out_features = out_features
        # unused by the RHS; kept for state_dict compatibility (:24-27)
        self.w = nn.Parameter(torch.eye(opt['hidden_dim']))
        self.d = nn.Parameter(torch.zeros(opt['hidden_dim']) + 1)
        self.alpha_sc = nn.Parameter(torch.ones(1))
        self.beta_sc = nn.Parameter(torch.ones(1))
        # set by integrator._OdeintAdjoint's backward while the weights are a constant of it
        # (adjoint_direct_ok): forward() then hands autograd the detached weights, so its
        # vector-Jacobian products form no weight gradient (the SDDMM) only to drop it
        self.adjoint_const_weights = False
        if opt.get('multi_modal', False):
            raise NotImplementedError("gnpde: multi_modal is broken in the reference (torch.nn.softmax, "
                                      "function_laplacian_diffusion.py:63) and out of scope")

    def _weights_tensor(self):
        blk = self.opt.get('block', 'constant')
        if blk == 'attention':
            w, tag = self.attention_weights, 'att_mean'
        elif blk in ('mixed', 'hard_attention'):
            w, tag = self.attention_weights, 'att'
        else:
            w, tag = self.edge_weight, 'w'
        if w is None:
            raise RuntimeError("LaplacianODEFunc: %s weights are not set for block=%r" % (tag, blk))
        return w, tag

    def supports_feature_padding(self):
        """Columns are independent (A x per column, x0 per column): the fused
        integrator may run on a zero-padded state (integrator._padded_width)."""
        return True

    def fixed_grid_backward_ok(self):
        """The fused discrete adjoint of a fixed-grid solve (integrator.
        _LaplacianFixedGridFn) covers gradients to the state, alpha_train and
        beta_train; a weight tensor that needs its own gradient (attention
        blocks training through the weights) keeps the per-RHS autograd path."""
        w, _ = self._weights_tensor()
        return not w.requires_grad

    def adjoint_direct_ok(self, adjoint_params):
        """The adjoint's augmented RHS may be evaluated by K1 launches (integrator.
        _LaplacianAdjointFn, _laplacian_aug) when the weights are not an adjoint
        parameter.  torchdiffeq's odeint_adjoint propagates into y0 and
        adjoint_params only (its forward runs under no_grad; the backward takes
        vector-Jacobian products with respect to those tensors alone), so a weight
        tensor the RHS closes over — AttODEblock's attention (src/block_transformer_
        attention.py:40-50), requiring grad in training — is a constant of the
        backward, exactly as upstream: its gradient from the ODE is dropped there too."""
        w, _ = self._weights_tensor()
        return all(p is not w for p in adjoint_params)

    def supports_node_layout(self):
        """Weights are per edge in COO order, x0 per node: the fixed-grid
        integrator may keep the state in the graph's locality numbering."""
        return True

    def _x0_like(self, x):
        """x0 in x's dtype and (padded) width, for the eager autograd path."""
        x0 = self.x0
        if x0.dtype != x.dtype:
            x0 = x0.to(x.dtype)
        if x0.shape[-1] != x.shape[-1]:
            x0 = self.stable_x0(x)
        return x0

    def graph_capture_state(self, x):
        """What a captured fused step reads (gnpde.integrator._capture_state):
        the device CSR + plan, the CSR-order weights and, with add_source, the
        stable x0 buffer — each refreshed in place from the current tensors."""
        g = self.graph_for(x)
        w, tag = self._weights_tensor()
        st = [g, self.csr_weights(g, w, tag)]
        if self.opt.get('add_source', False):
            st.append(self.stable_x0(x))
        return st

    def sparse_multiply(self, x):
        """A x (src/function_laplacian_diffusion.py:39-58) — K1 without the epilogue."""
        g = self.graph_for(x)
        w, tag = self._weights_tensor()
        return ops.spmm_rhs(g, self.csr_weights(g, w, tag), x, rhs=False)

    # f(x) = sigma(alpha)(A - I) x [+ beta x0] is affine in x with the weights fixed for a solve
    # (every block: constant, attention / hard_attention / mixed weights are computed once per forward)
    affine = True
    # rhs_stage takes Stage.dense (the plain-weight K1): an adaptive solve in the Krylov basis may fold
    # its dense output into the steps' last launch (integrator.DENSE_FOLD)
    fold_dense = True

    def rhs_stage(self, t, x, stage, linear=False):
        """forward(t, x) with the solver's stage combination fused into the K1
        epilogue (gnpde.integrator, no-grad fixed-grid solvers).  linear=True
        evaluates the linear part sigma(alpha)(A - I) x alone (no source term):
        the adaptive solvers' affine stage derivatives (Stage.f_lin)."""
        if self.nfe > self.opt["max_nfe"]:
            raise MaxNFEException
        self.nfe += 1
        g = self.graph_for(x)
        w, tag = self._weights_tensor()
        add_source = bool(self.opt.get('add_source', False)) and not linear
        x0 = self.stable_x0(x) if add_source else None
        ops.spmm_rhs(g, self.csr_weights(g, w, tag), x, x0=x0, alpha=self.alpha_train.detach(),
                     beta=self.beta_train.detach(), rhs=True, alpha_sigmoid=not self.opt.get('no_alpha_sigmoid', False),
                     add_source=add_source, stage=stage)

    def forward(self, t, x):  # the t param is needed by the ODE solver.
        if self.nfe > self.opt["max_nfe"]:
            raise MaxNFEException
        self.nfe += 1
        g = self.graph_for(x)
        w, tag = self._weights_tensor()
        w_csr = self.csr_weights(g, w, tag)
        add_source = bool(self.opt.get('add_source', False))
        if add_source and self.x0 is None:
            raise RuntimeError("LaplacianODEFunc: add_source needs x0 (ODEblock.set_x0)")
        alpha_sigmoid = not self.opt.get('no_alpha_sigmoid', False)
        x0 = self._x0_like(x) if add_source else None
        if x.dtype == torch.bfloat16:
            # bf16 storage (configs[3]): inference only — the backward kernels are fp32
            if torch.is_grad_enabled() and (x.requires_grad or self.alpha_train.requires_grad):
                raise NotImplementedError("gnpde: bf16 state is inference-only; run under torch.no_grad()")
            return ops.spmm_rhs(g, w_csr, x, x0=x0, alpha=self.alpha_train.detach(), beta=self.beta_train.detach(),
                                rhs=True, alpha_sigmoid=alpha_sigmoid, add_source=add_source)
        w_src = w.detach() if self.adjoint_const_weights else w
        return _LaplacianRHS.apply(x, self.alpha_train, self.beta_train, w_src, g, w_csr,
                                   lambda: self.csr_weights(g, w, tag, transpose=True), x0, alpha_sigmoid,
                                   add_source)
