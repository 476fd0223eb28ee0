"""Drop-in ConstantODEblock (reference src/block_constant.py:5-63).

``forward(x, graph_data, y=None)``: prepare the graph once (cached), then
integrate ``odefunc`` from t[0] to t[1] with the reference's method /
step_size / tolerances and return the state at t[1].
"""
import torch

from .base_classes import ODEblock
from .integrator import odeint, odeint_adjoint


class ConstantODEblock(ODEblock):
    def __init__(self, odefunc, regularization_fns, opt, device, t=torch.tensor([0, 1])):
        super(ConstantODEblock, self).__init__(odefunc, regularization_fns, opt, device, t)
        self.device = device
        self.odefunc = self._new_odefunc(odefunc, opt, device)  # the integrated copy (src/block_constant.py:11)
        self.train_integrator = odeint_adjoint if opt.get('adjoint', False) else odeint
        self.test_integrator = odeint
        self.set_tol()

    def forward(self, x, graph_data, y=None):
        self.reset_graph_data(graph_data, x.dtype, y)
        return self._integrate(x, dict(step_size=self.opt.get('step_size'), max_iters=self.opt.get('max_iters')))

    def __repr__(self):
        return self.__class__.__name__ + '( Time Interval ' + str(self.t[0].item()) + ' -> ' + \
            str(self.t[1].item()) + ")"
