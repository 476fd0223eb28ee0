"""Drop-in registry (reference src/model_configurations.py:17-44): the plugin
point ``GNN.__init__`` uses (src/GNN.py:12-15).

Built here: block 'constant', 'attention', 'mixed',
'hard_attention'; function 'laplacian', 'transformer'.  The other names the
reference registers are out of scope ('rewire_attention', 'GAT') and raise
NotImplementedError naming the reason, rather than silently falling back to a
different model.
"""
from .block_constant import ConstantODEblock
from .block_mixed import MixedODEblock
from .block_transformer_hard_attention import HardAttODEblock
from .block_transformer_attention import AttODEblock
from .function_laplacian_diffusion import LaplacianODEFunc
from .function_transformer_attention import ODEFuncTransformerAtt


class BlockNotDefined(Exception):
    pass


class FunctionNotDefined(Exception):
    pass


_PENDING_BLOCKS = {
    'rewire_attention': 'out of scope (graph surgery between forwards, SURVEY §2 row 9)',
}


def set_block(opt):
    ode_str = opt['block']
    if ode_str == 'mixed':
        return MixedODEblock
    if ode_str == 'attention':
        return AttODEblock
    if ode_str == 'hard_attention':
        return HardAttODEblock
    if ode_str == 'constant':
        return ConstantODEblock
    if ode_str in _PENDING_BLOCKS:
        raise NotImplementedError("gnpde: block %r is %s" % (ode_str, _PENDING_BLOCKS[ode_str]))
    raise BlockNotDefined


def set_function(opt):
    ode_str = opt['function']
    if ode_str == 'laplacian':
        return LaplacianODEFunc
    if ode_str == 'transformer':
        return ODEFuncTransformerAtt
    if ode_str == 'GAT':
        raise NotImplementedError("gnpde: function 'GAT' is out of scope (not named by the north star, SURVEY §2 "
                                  "row 10)")
    raise FunctionNotDefined
