"""Drop-in ODEFuncTransformerAtt and SpGraphTransAttentionLayer
(reference src/function_transformer_attention.py:9-270).

Per RHS evaluation the reference projects Q/K/V, gathers q[src] and k[dst],
forms an [B,h,E,E] score matmul, runs utils.softmax and densifies the
head-mean attention into [B,N,N] for a dense matmul.  Here one RHS is:

1. node scores — reference ``scaled_dot`` (the fork's global key sum,
   :249 = ``q_src . (sum_e' k_dst(e')) / sqrt(dk)``) needs no
   per-edge work at all: an indegree-weighted column sum of x (fp64), a tiny
   key projection, and one fp64 GEMV per node (gnpde_ref_scores_f32).  The
   per-edge modes (``score_mode='per_edge'`` scaled_dot = upstream GRAND, and
   exp_kernel / cosine_sim / pearson, :246-259) project Q|K with the MFMA
   kernel (gnpde_linear_f32);
2. norm_idx 1: destination-grouped softmax statistics (max, 1/sum-exp)
   over the CSC (K2, gnpde_seg_softmax_f32);
3. head-mean softmax weights in aggregation-CSR order: for norm_idx 0 the
   edge-block segmented-softmax kernel K2 computes them straight from the
   scores (SDDMM + segmented max/sum-exp + head mean in one pass, no [E,h]
   tensor); for norm_idx 1 an edge-parallel pass over the statistics of
   step 2 (gnpde_attn_weights_f32); then the K1 gather-aggregate with the RHS /
   Runge-Kutta epilogue fused (gnpde_spmm_rhs_f32).  With the fork scaled_dot
   and norm_idx 0 every score of a source group is equal, so the weights are
   1/outdeg for any x: computed once per graph.

V and Wout are dead when ``mix_features=False`` (:33-41) and are never
computed; the parameters exist for state_dict compatibility.  Settings the
fork cannot execute (``mix_features`` :23-31, ``square_plus`` :264,
``multi_modal`` :171/222, beltrami+exp_kernel :164-167) raise
NotImplementedError.  ``reweight_attention`` is a no-op in the fork (the
layer's ``edge_weights`` is captured as None at construction, :15 / :261) and
is a no-op here.

Gradients: with autograd recording, the layer's forward
is ``_EdgeAttention`` — the same forward kernels, plus a backward made of graph
passes (backward.hip): edge-softmax backward per group, then for the fork's
scaled_dot the node-score / key-sum chain rule (segment sums, fp64 weighted
column sums, a few [att, C] products) and for the per-edge scaled_dot two K1
aggregations per head (q side over the CSR, k side over the CSC) and the
projection backward (MFMA projections for d/dx and d/dW, gnpde_linear_wgrad_f32).  The
transformer ODEFunc then composes it with the Laplacian RHS autograd
(function_laplacian_diffusion._LaplacianRHS), whose weight gradient is an
SDDMM.  exp_kernel / cosine_sim / pearson: one pass per side over the grouped
CSR / CSC turns dL/ds into dL/dq and dL/dk (gnpde_score_grad_f32, exp_kernel
also into dL/d output_var and dL/d lengthscale), then the same projection
backward.  Every gradient is pinned by fixtures of the reference's own fp64
autograd (tests/golden/grad_*.npz, tests/test_gpu_grad_golden.py).
"""
import torch
from torch import nn

from . import ops
from .base_classes import ODEFunc, _tensor_key
from .utils import MaxNFEException


def _check_supported(opt):
    if opt.get('mix_features', False):
        raise NotImplementedError("gnpde: mix_features=True is broken in the reference "
                                  "(function_transformer_attention.py:29-31 uses a tuple as a tensor)")
    if opt.get('square_plus', False):
        raise NotImplementedError("gnpde: square_plus is broken in the reference (utils.squareplus called "
                                  "without num_nodes, :264) and not implemented")
    if opt.get('multi_modal', False):
        raise NotImplementedError("gnpde: multi_modal is broken in the reference and out of scope")
    if opt.get('beltrami', False) and opt.get('attention_type', 'scaled_dot') == 'exp_kernel':
        raise NotImplementedError("gnpde: the beltrami exp_kernel branch slices nodes instead of features in the "
                                  "reference (:166-167) and is not implemented")


def _needs_grad(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


class _EdgeAttention(torch.autograd.Function):
    """attention [B,E,h] (COO) = SpGraphTransAttentionLayer.forward's first
    output as a function of (x, Wq, bq, Wk, bk[, output_var, lengthscale]);
    backward in graph passes."""

    @staticmethod
    def forward(ctx, x, Wq, bq, Wk, bk, ov, ls, layer, g, norm_idx):
        ns, m, rl = layer.scores_and_stats(g, x.detach(), norm_idx)
        att = ops.edge_attention(g, ns, m, rl, norm_idx)
        ctx.save_for_backward(x, Wq, bq, Wk, bk, att)
        ctx.layer, ctx.g, ctx.norm_idx, ctx.ns = layer, g, norm_idx, ns
        ctx.p_shapes = (None if ov is None else (ov.shape, ov.dtype), None if ls is None else (ls.shape, ls.dtype))
        return att

    @staticmethod
    def backward(ctx, g_att):
        x, Wq, bq, Wk, bk, att = ctx.saved_tensors
        g, ns, norm_idx = ctx.g, ctx.ns, ctx.norm_idx
        grouped = g.csr if norm_idx == 0 else g.csc
        gs = ops.softmax_backward(grouped, att, g_att.float())
        g_ov = g_ls = None
        if ns.mode == ops._lib.SCORE_UNIFORM:
            # every score of a softmax group is the same node score: the attention does not move
            grads = (torch.zeros_like(x), torch.zeros_like(Wq), torch.zeros_like(bq), torch.zeros_like(Wk),
                     torch.zeros_like(bk))
        elif ns.mode == ops._lib.SCORE_REFERENCE:
            grads = _reference_score_backward(g, ns, gs, x.detach(), Wq.detach(), bq.detach(), Wk.detach(),
                                              bk.detach())
        elif ns.mode == ops._lib.SCORE_DOT:
            grads = _dot_score_backward(g, ns, gs, x.detach(), Wq.detach(), Wk.detach())
        else:
            grads, gp = _edge_score_backward(g, ns, gs, x.detach(), Wq.detach(), Wk.detach())
            if gp is not None:
                (so, do), (sl, dl) = ctx.p_shapes
                g_ov, g_ls = gp[0].reshape(so).to(do), gp[1].reshape(sl).to(dl)
        return grads + (g_ov, g_ls, None, None, None)


def _reference_score_backward(g, ns, gs, x, Wq, bq, Wk, bk):
    """Chain rule of the fork's scaled_dot (function_transformer_attention.py:249):
    s[e,h] = cs[src(e),h], cs[n,h] = q_{n,h} . S_h / sqrt(dk), q = Wq x + bq,
    S = Wk xbar + E bk, xbar = sum_n indeg(n) x_n.  Graph passes in HIP; the
    [att, C]-sized products in fp64 torch."""
    B, N, H, dk = g.B, g.N, ns.heads, ns.dk
    att_dim = H * dk
    C = x.shape[-1]
    inv = 1.0 / float(dk) ** 0.5
    gcs = ops.segment_sum(g.csr, gs)                           # [R,H]: edges gather the score of their source
    xbar = ops.wcolsum(x, B, N, g.indeg.double().view(-1, 1))[:, 0, :]    # [B,C+1]
    y = ops.wcolsum(x, B, N, gcs)                              # [B,H,C+1]
    Wq64, bq64, Wk64, bk64 = Wq.double(), bq.double(), Wk.double(), bk.double()
    S = xbar[:, :C] @ Wk64.t() + xbar[:, C:] * bk64            # [B,att]
    Sh = S.view(B, H, dk)
    Wqh = Wq64.view(H, dk, C)
    U = inv * torch.einsum('hdc,bhd->bch', Wqh, Sh)            # [B,C,H]
    gU = y[:, :, :C].transpose(1, 2)                           # [B,C,H]
    gv = y[:, :, C]                                            # [B,H]
    g_Wq = inv * torch.einsum('bhd,bch->hdc', Sh, gU).reshape(att_dim, C)
    g_bq = inv * torch.einsum('bhd,bh->hd', Sh, gv).reshape(att_dim)
    gS = inv * (torch.einsum('hdc,bch->bhd', Wqh, gU) + bq64.view(H, dk)[None] * gv[:, :, None])
    gS = gS.reshape(B, att_dim)
    g_Wk = gS.t() @ xbar[:, :C]
    g_bk = gS.t() @ xbar[:, C]
    gxbar = gS @ Wk64                                          # [B,C]
    gx = ops.score_input_grad(gcs, U, g.indeg, gxbar, B, N, C).view(x.shape)
    return (gx, g_Wq.to(Wq.dtype), g_bq.to(bq.dtype), g_Wk.to(Wk.dtype), g_bk.to(bk.dtype))


def _dot_score_backward(g, ns, gs, x, Wq, Wk):
    """Per-edge scaled_dot s[e,h] = q[src,h] . k[dst,h] / sqrt(dk): per head, g_q
    aggregates g_s k[dst] over the CSR and g_k aggregates g_s q[src] over the
    CSC (K1 with per-head weights), then the projection backward."""
    H, dk = ns.heads, ns.dk
    inv = 1.0 / float(dk) ** 0.5
    R = g.R
    xr = x.reshape(R, -1)
    gqk = torch.empty(R, 2 * H * dk, dtype=torch.float32, device=x.device)
    for h in range(H):
        cols = slice(h * dk, (h + 1) * dk)
        kh = ns.k[:, cols].contiguous()
        qh = ns.q[:, cols].contiguous()
        gqk[:, cols] = ops.spmm_rhs(g, ops.gather_head(g.csr, gs, h, inv), kh, rhs=False)
        gqk[:, H * dk + h * dk:H * dk + (h + 1) * dk] = ops.spmm_rhs(g, ops.gather_head(g.csc, gs, h, inv), qh,
                                                                     rhs=False, transpose=True)
    W = torch.cat([Wq, Wk], 0)                                 # [2att, C]
    gx, _ = ops.linear(gqk, W.t().contiguous())                # gx = [g_q | g_k] [Wq; Wk]
    gW = ops.linear_wgrad(gqk, xr)                             # [2att, C] = gqk^T x on the matrix cores
    gb = gqk.sum(0)
    att_dim = H * dk
    return (gx.view(x.shape), gW[:att_dim], gb[:att_dim], gW[att_dim:], gb[att_dim:])


def _edge_score_backward(g, ns, gs, x, Wq, Wk):
    """exp_kernel / cosine_sim / pearson (function_transformer_attention.py:246-259):
    dL/dq over the aggregation CSR (edges grouped by source) and dL/dk over the
    CSC (grouped by destination) in one pass each (gnpde_score_grad_f32), then
    the projection backward as for the per-edge scaled_dot.  exp_kernel also
    returns dL/d(output_var), dL/d(lengthscale)."""
    with_p = ns.mode == ops._lib.SCORE_EXP_KERNEL
    if with_p:
        gq, gov, gls = ops.score_grad(g.csr, 0, ns, gs, with_params=True)
    else:
        gq = ops.score_grad(g.csr, 0, ns, gs)
    gk = ops.score_grad(g.csc, 1, ns, gs)
    gqk = torch.cat([gq, gk], 1)
    xr = x.reshape(g.R, -1)
    W = torch.cat([Wq, Wk], 0)
    gx, _ = ops.linear(gqk, W.t().contiguous())                # gx = [g_q | g_k] [Wq; Wk]
    gW = ops.linear_wgrad(gqk, xr)
    gb = gqk.sum(0)
    att_dim = ns.heads * ns.dk
    grads = (gx.view(x.shape), gW[:att_dim], gb[:att_dim], gW[att_dim:], gb[att_dim:])
    return grads, ((gov, gls) if with_p else None)


class SpGraphTransAttentionLayer(nn.Module):
    """src/function_transformer_attention.py:65-270 (standard branch)."""

    def __init__(self, in_features, out_features, opt, device, concat=True, edge_weights=None):
        super(SpGraphTransAttentionLayer, self).__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = opt.get('leaky_relu_slope', 0.2)
        self.concat = concat
        self.device = device
        self.opt = opt
        self.h = int(opt['heads'])
        self.edge_weights = edge_weights
        self.attention_dim = opt.get('attention_dim', out_features)
        assert self.attention_dim % self.h == 0, \
            "Number of heads ({}) must be a factor of the dimension size ({})".format(self.h, self.attention_dim)
        self.d_k = self.attention_dim // self.h
        _check_supported(opt)
        if opt.get('attention_type', 'scaled_dot') == "exp_kernel":
            self.output_var = nn.Parameter(torch.ones(1))
            self.lengthscale = nn.Parameter(torch.ones(1))
        self.Q = nn.Linear(in_features, self.attention_dim)
        self.init_weights(self.Q)
        self.V = nn.Linear(in_features, self.attention_dim)
        self.init_weights(self.V)
        self.K = nn.Linear(in_features, self.attention_dim)
        self.init_weights(self.K)
        self.activation = nn.Sigmoid()
        self.Wout = nn.Linear(self.d_k, in_features)
        self.init_weights(self.Wout)
        self._graph = None
        self._graph_key = None
        self._uniform = None  # (graph, NodeScores, m, rl, csr weights) for the uniform fast path
        self._wcat = None     # (param versions, ([Wq;Wk], [bq;bk]))

    def init_weights(self, m):
        """Constant 1e-5 init (:153-157)."""
        if type(m) == nn.Linear:
            nn.init.constant_(m.weight, 1e-5)

    @property
    def score_mode(self):
        return self.opt.get('attention_score_mode', 'reference')

    def _score_params(self):
        if self.opt.get('attention_type', 'scaled_dot') == 'exp_kernel':
            # p0 = output_var, p1 = lengthscale: read once per call (host sync of 2 scalars)
            return float(self.output_var.detach()), float(self.lengthscale.detach())
        return 1.0, 1.0

    def graph_for(self, x, edge):
        key = (_tensor_key(edge), int(x.shape[1]))
        if self._graph is None or key != self._graph_key:
            self._graph = ops.GraphCSR(edge, int(x.shape[1]), chunk=self.opt.get('gnpde_chunk'))
            self._graph_key = key
        return self._graph

    def is_uniform(self, norm_idx):
        """Fork scaled_dot + source-grouped softmax: all scores of a group are equal,
        so the attention is 1/outdeg whatever x — graph-only, cached."""
        return (self.score_mode == 'reference' and norm_idx == 0 and
                self.opt.get('attention_type', 'scaled_dot') == 'scaled_dot')

    def scores_and_stats(self, g, x, norm_idx):
        """(NodeScores, m, rl) for this RHS evaluation."""
        if self.is_uniform(norm_idx):
            if self._uniform is None or self._uniform[0] is not g:
                ns = ops.uniform_scores(self.h)
                m, rl = ops.softmax_stats(g, ns, 0)
                self._uniform = (g, ns, m, rl, ops.attn_weights(g, ns, m, rl, 0))
            return self._uniform[1:4]
        ns = self.node_scores(g, x)
        m, rl = ops.softmax_stats(g, ns, norm_idx)
        return ns, m, rl

    def uniform_weights(self, g):
        self.scores_and_stats(g, None, 0)
        return self._uniform[4]

    def uses_wcat(self):
        """Per-edge score modes project Q|K with one fused MFMA GEMM over [Wq; Wk]."""
        return self.score_mode != 'reference' or self.opt.get('attention_type', 'scaled_dot') != 'scaled_dot'

    def wcat(self):
        """([Wq; Wk], [bq; bk]) cached per parameter version."""
        key = tuple(_tensor_key(t) for t in (self.Q.weight, self.Q.bias, self.K.weight, self.K.bias))
        if self._wcat is None or self._wcat[0] != key:
            self._wcat = (key, (torch.cat([self.Q.weight.detach(), self.K.weight.detach()], 0).contiguous(),
                                torch.cat([self.Q.bias.detach(), self.K.bias.detach()], 0).contiguous()))
        return self._wcat[1]

    def node_scores(self, g, x):
        p0, p1 = self._score_params()
        wcat = self.wcat() if self.uses_wcat() else None
        return ops.node_scores(g, x, self.Q.weight.detach(), self.Q.bias.detach(), self.K.weight.detach(),
                               self.K.bias.detach(), self.h, self.opt.get('attention_type', 'scaled_dot'),
                               self.score_mode, p0, p1, wcat=wcat)

    def forward(self, x, edge, y=None):
        """Returns (attention [B,E,h], (None, None)): the per-edge softmax
        attention of :265-266 in COO order.  ``values`` (V(x), prods) is not
        materialised (dead for mix_features=False)."""
        g = self.graph_for(x, edge)
        norm_idx = int(self.opt['attention_norm_idx'])
        ov = getattr(self, 'output_var', None)
        ls = getattr(self, 'lengthscale', None)
        if _needs_grad(x, self.Q.weight, self.Q.bias, self.K.weight, self.K.bias, ov, ls):
            att = _EdgeAttention.apply(x, self.Q.weight, self.Q.bias, self.K.weight, self.K.bias, ov, ls, self, g,
                                       norm_idx)
            return att, (None, None)
        ns, m, rl = self.scores_and_stats(g, x, norm_idx)
        return ops.edge_attention(g, ns, m, rl, norm_idx), (None, None)

    def __repr__(self):
        return self.__class__.__name__ + ' (' + str(self.in_features) + ' -> ' + str(self.out_features) + ')'


class ODEFuncTransformerAtt(ODEFunc):
    """src/function_transformer_attention.py:9-62."""

    def __init__(self, in_features, out_features, opt, device):
        super(ODEFuncTransformerAtt, self).__init__(opt, device)
        self.in_features = in_features
        self.out_features = out_features
        self.multihead_att_layer = SpGraphTransAttentionLayer(in_features, out_features, opt, device,
                                                              edge_weights=self.edge_weight)
        if device is not None:
            self.multihead_att_layer = self.multihead_att_layer.to(device)
        self.y = None

    def multiply_attention(self, x, attention, v=None):
        """A_mean x with attention [B,E,h] given explicitly (:20-42)."""
        g = self.graph_for(x)
        w = g.gather_weights(attention.detach().float())
        return ops.spmm_rhs(g, w, x, rhs=False)

    def rhs_stage(self, t, x, stage):
        """forward(t, x) with the solver's stage combination fused into the
        aggregation epilogue (gnpde.integrator, no-grad fixed-grid solvers)."""
        self._rhs(x, stage)

    def graph_capture_state(self, x):
        """What a captured fused step reads (gnpde.integrator._capture_state):
        the device CSR / CSC + plans, the layer's cached operands (the 1/outdeg
        weights of the uniform case, or the concatenated [Wq; Wk] projection)
        and, with add_source, the stable x0 buffer."""
        g = self.graph_for(x)
        lay = self.multihead_att_layer
        st = [g]
        if lay.is_uniform(int(self.opt['attention_norm_idx'])):
            lay.uniform_weights(g)
            st.append(lay._uniform)
        elif lay.uses_wcat():
            st.append(lay.wcat())
        if self.opt.get('add_source', False):
            st.append(self.stable_x0(x))
        return st

    def supports_node_layout(self):
        """The graph's locality numbering (ops.NodeLayout) for fixed-grid solves: every
        operand of the scaled_dot RHS is per node (x, q, k, node scores) or per edge
        in COO order, and a renumbering relabels them consistently, so the scores,
        the softmax groups and the aggregation are the same.  Bit-identical for the
        weights that are row-local in the fused kernels (the fork's 1/outdeg weights
        under source-grouped softmax — BLEND — and the per-edge scores under
        source-grouped softmax: each row scores and sums its own edges in COO
        order); the key sum of the fork's scores (fp64, row-tile order) and the
        destination statistics (packed CSC edge blocks) are summed in another order,
        within fp64 / fp32 rounding (tests/test_gpu_layout.py).  Other attention
        types keep the user numbering."""
        lay = self.multihead_att_layer
        return lay.is_uniform(int(self.opt['attention_norm_idx'])) or \
            self.opt.get('attention_type', 'scaled_dot') == 'scaled_dot'

    def supports_feature_padding(self):
        """With the fork's scaled_dot under source-grouped softmax the weights do
        not depend on x (1/outdeg), so columns are independent and the fused
        integrator may pad the state (integrator._padded_width); score modes
        read Q/K over all C columns and may not."""
        return self.multihead_att_layer.is_uniform(int(self.opt['attention_norm_idx'])) and \
            not self.opt.get('add_source', False)

    def forward(self, t, x):  # t is needed when called by the integrator
        return self._rhs(x, None)

    def _rhs(self, x, stage):
        if self.nfe > self.opt["max_nfe"]:
            raise MaxNFEException
        self.nfe += 1
        g = self.graph_for(x)
        lay = self.multihead_att_layer
        if stage is None and _needs_grad(x, self.alpha_train, self.beta_train, lay.Q.weight, lay.Q.bias,
                                         lay.K.weight, lay.K.bias, getattr(lay, 'output_var', None),
                                         getattr(lay, 'lengthscale', None)):
            return self._rhs_autograd(g, x)
        norm_idx = int(self.opt['attention_norm_idx'])
        add_source = bool(self.opt.get('add_source', False))
        if add_source and self.x0 is None:
            raise RuntimeError("ODEFuncTransformerAtt: add_source needs x0 (ODEblock.set_x0)")
        # fused stages (and their captured graphs) read a stable x0 buffer (ODEFunc.stable_x0)
        x0 = (self.stable_x0(x) if stage is not None else self.x0) if add_source else None
        if x0 is not None and x0.dtype != x.dtype:
            x0 = x0.to(x.dtype)
        kw = dict(x0=x0, alpha=self.alpha_train.detach(), beta=self.beta_train.detach(),
                  rhs=True, alpha_sigmoid=not self.opt.get('no_alpha_sigmoid', False), add_source=add_source,
                  stage=stage)
        if lay.is_uniform(norm_idx):
            return ops.spmm_rhs(g, lay.uniform_weights(g), x, **kw)
        if x.dtype == torch.bfloat16:
            # bf16 storage: the per-edge scores' projection reads the bf16 state itself
            # (gnpde_linear_bf16, the same bits as from an fp32 copy); the fork's reference
            # scores (fp64 key sum and node scores) from an fp32 copy; weights precomputed,
            # bf16 aggregation
            ref = lay.score_mode == 'reference' and self.opt.get('attention_type', 'scaled_dot') == 'scaled_dot'
            ns = lay.node_scores(g, x.float() if ref else x)
            m, rl = ops.softmax_stats(g, ns, 1) if norm_idx == 1 else (None, None)
            # per-edge scaled_dot under source-grouped softmax: the fused pass over the bf16
            # state (gnpde_attn_dot_rhs_bf16); otherwise K2 weights + the bf16 K1
            return ops.attn_rhs(g, ns, m, rl, norm_idx, x, fuse=not ref and norm_idx == 0, **kw)
        ns = lay.node_scores(g, x)
        # destination-grouped softmax needs its statistics over the CSC first
        # (attn_rhs computes them: packed records for the fork's two-head
        # scores); source-grouped weights come straight from the scores (K2)
        return ops.attn_rhs(g, ns, None, None, norm_idx, x, **kw)

    def _rhs_autograd(self, g, x):
        """Training forward: attention [B,E,h] through _EdgeAttention, then the
        Laplacian RHS autograd with those weights (head mean), so gradients
        reach x (both paths), alpha, beta and the Q/K parameters."""
        from .function_laplacian_diffusion import _LaplacianRHS
        att, _ = self.multihead_att_layer(x, self.edge_index)
        add_source = bool(self.opt.get('add_source', False))
        if add_source and self.x0 is None:
            raise RuntimeError("ODEFuncTransformerAtt: add_source needs x0 (ODEblock.set_x0)")
        x0 = self.x0 if add_source else None
        if x0 is not None and x0.dtype != torch.float32:
            x0 = x0.float()
        ad = att.detach()
        return _LaplacianRHS.apply(x, self.alpha_train, self.beta_train, att, g, g.gather_weights(ad),
                                   lambda: g.gather_weights(ad, transpose=True), x0,
                                   not self.opt.get('no_alpha_sigmoid', False), add_source)

    def __repr__(self):
        return self.__class__.__name__ + ' (' + str(self.in_features) + ' -> ' + str(self.out_features) + ')'
