"""Identity keys for the per-module caches of derived device data (CSR, plans,
CSR-order weights, stable x0 buffers, captured step graphs)."""


class _TensorKey(object):
    """Identity key of a tensor for the derived-data caches: the tensor itself
    (held, so no other tensor can be allocated at its address while the key
    lives), its version counter (in-place updates) and its shape / dtype.
    Equal only for the SAME tensor object in the same version."""
    __slots__ = ('t', 'version', 'meta')

    def __init__(self, t):
        self.t = t
        self.version = t._version
        self.meta = (tuple(t.shape), t.dtype, str(t.device))

    def __eq__(self, other):
        return isinstance(other, _TensorKey) and other.t is self.t and other.version == self.version and \
            other.meta == self.meta

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash((id(self.t), self.version))


def _tensor_key(t):
    if t is None:
        return None
    return _TensorKey(t)
