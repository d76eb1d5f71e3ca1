"""The LeNet training step as two native dispatches (``csrc/lenet_fused.hip``).

Reference: the task3 loop (codes/task3/model.py:50-64) on ``Net``
(codes/task1/pytorch/model.py:12-35): ``outputs = model(x); loss = CE(outputs, y);
zero_grad(); loss.backward(); [average_gradients]; step()``.

:class:`FusedLeNetStep` keeps that contract — same parameters (the Program's flat fp32
buffer), same optimiser state, same DDP averaging — but runs it as

* ``lenet_sample_kernel``: one workgroup per sample, the whole forward and backward of
  the sample in LDS (no per-layer launches, no autograd graph, no ATen kernels);
* ``lenet_grad_kernel``: the batch reduction of every gradient into ``flat.grad`` and, on
  one rank, the SGD update fused into the same dispatch;

and with ``DDP``: the bucket all-reduce of ``flat.grad`` (RCCL or the xGMI kernel) and the
fused SGD kernel.  Nothing allocates or synchronises, so the step is hipGraph-capturable at
any world size.  The CPU (and ``backend="torch"``) falls back to the autograd step.
"""
from __future__ import annotations

import torch

from dmlab.models.lenet import Net


class FusedLeNetStep:
    def __init__(self, net: Net, optimizer=None, ddp=None):
        if not isinstance(net, Net):
            raise TypeError("FusedLeNetStep needs the reference LeNet (dmlab.models.Net)")
        self.net, self.opt, self.ddp = net, optimizer, ddp
        flat = net.flat
        order = [net.fc2.weight, net.fc2.bias, net.fc1.weight, net.fc1.bias,
                 net.conv2.weight, net.conv2.bias, net.conv1.weight, net.conv1.bias]
        self.offsets = [int(flat.offsets[flat.index_of(p)]) for p in order]
        self.weights = [net.conv1.weight, net.conv1.bias, net.conv2.weight, net.conv2.bias,
                        net.fc1.weight, net.fc1.bias, net.fc2.weight, net.fc2.bias]
        self._ws = {}
        self.loss = torch.zeros((), device=flat.device, dtype=torch.float32)
        # running sum of the step losses, accumulated on the device by the gradient kernel
        # (a training loop reads it every `log_every` steps without a per-step sync)
        self.loss_sum = torch.zeros(1, device=flat.device, dtype=torch.float32)

    def _workspace(self, B):
        w = self._ws.get(B)
        if w is None:
            from dmlab.ops._native import lib

            L = lib()
            dev = self.net.flat.device
            w = (torch.empty(B * L.lenet_record_floats(), device=dev),
                 torch.empty(B * L.lenet_slab_floats(), device=dev),
                 torch.empty(B, device=dev))
            self._ws[B] = w
        return w

    def _fused_sgd(self):
        from dmlab.optim import SGD

        opt = self.opt
        return (isinstance(opt, SGD) and opt.flat is self.net.flat and
                (self.ddp is None or not self.ddp.comm_active))

    def __call__(self, x: torch.Tensor, y: torch.Tensor, cursor=None) -> torch.Tensor:
        """One step on batch (x, y); or, with ``cursor`` (:class:`dmlab.data.DeviceCursor`),
        on the cursor's next batch of the device-resident dataset ``(x, y)`` = (all images,
        all labels): the sample kernel gathers its rows through the epoch order and the
        gradient kernel advances the cursor, so a captured graph walks the epoch."""
        if not x.is_cuda or self.net.backend == "torch":
            if cursor is not None:
                raise ValueError("the device cursor needs the native GPU step")
            return self._autograd_step(x, y)
        from dmlab.ops._native import lib

        flat = self.net.flat
        B = cursor.loader.batch_size if cursor is not None else x.shape[0]
        rec, slab, rowloss = self._workspace(B)
        x = x.contiguous()
        ix = {} if cursor is None else dict(sidx=cursor.order, cursor=cursor.cursor, batch=B)
        ix["loss_sum"] = self.loss_sum
        if self._fused_sgd():
            opt = self.opt
            opt.step_count += 1
            lib().lenet_fused_step(x, y, self.weights, rec, slab, rowloss, flat.grad, self.offsets,
                                   flat.data, opt.buf, opt.lr, opt.momentum, opt.dampening,
                                   opt.weight_decay, opt.grad_scale, opt.nesterov,
                                   opt.step_count == 1, self.loss, **ix)
            flat.mark_updated()
            flat.mark_grads_consumed()
            return self.loss
        lib().lenet_fused_step(x, y, self.weights, rec, slab, rowloss, flat.grad, self.offsets,
                               None, None, 0.0, 0.0, 0.0, 0.0, 1.0, False, False, self.loss, **ix)
        flat.grad_valid = True
        if self.ddp is not None:
            self.ddp.reduce_now()
        if self.opt is not None:
            self.opt.step()
        return self.loss

    def _autograd_step(self, x, y):
        from dmlab.nn import cross_entropy

        model = self.ddp if self.ddp is not None else self.net
        loss = cross_entropy(model(x), y)
        if self.opt is not None:
            self.opt.zero_grad()
        loss.backward()
        if self.opt is not None:
            self.opt.step()
        return loss.detach()
