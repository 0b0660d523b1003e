"""On-policy serial trainer (RL/trainer/on_serial_trainer.py:14-122) for PPO / POLYC.

Same loop: sample_with_replay_format() -> model_update(samples) -> (tb, global_iteration) ->
log / save / evaluate, until global_iteration reaches max_iteration. Device boundary: the
sampler's batch is already in HBM (no `.cuda()` copies, :60-62) and the networks stay on the
sampler's device instead of moving around each phase (ModuleOnDevice, :63,84).
"""
__all__ = ["OnSerialTrainer"]

import os
import time
from math import inf

import torch

from ..utils import dist as D
from ..utils.common_utils import ModuleOnDevice
from ..utils.log_data import LogData
from ..utils.tensorboard_setup import add_scalars, make_writer, tb_tags


class OnSerialTrainer:
    def __init__(self, alg, sampler, evaluator, **kwargs):
        self.alg = alg
        self.sampler = sampler
        self.evaluator = evaluator
        self.networks = self.alg.networks
        self.sampler.networks = self.networks
        if self.evaluator is not None:
            self.evaluator.networks = self.networks
        if kwargs.get("ini_network_dir") is not None:
            self.networks.load_state_dict(torch.load(kwargs["ini_network_dir"], weights_only=True))
        D.broadcast_module(self.networks)
        self.max_iteration = kwargs["max_iteration"]
        self.log_save_interval = kwargs["log_save_interval"]
        self.apprfunc_save_interval = kwargs["apprfunc_save_interval"]
        self.eval_interval = kwargs["eval_interval"]
        self.save_folder = kwargs["save_folder"]
        self.is_main = D.rank() == 0
        self.writer = make_writer(self.save_folder, flush_secs=20)
        add_scalars({tb_tags["alg_time"]: 0, tb_tags["sampler_time"]: 0}, self.writer, 0)
        self.writer.flush()
        self.sampler_tb_dict = LogData()
        self.best_tar = -inf
        self.global_iteration = 0
        self.use_gpu = kwargs.get("use_gpu", torch.cuda.is_available())
        self.sample_device = getattr(self.sampler, "device", "cpu")
        self.start_time = time.time()

    def step(self):
        with ModuleOnDevice(self.networks, self.sample_device):
            samples, sampler_tb_dict = self.sampler.sample_with_replay_format()
        self.sampler_tb_dict.add_average(sampler_tb_dict)
        self.networks.train()
        alg_tb_dict, self.global_iteration = self.alg.model_update(samples)
        self.networks.eval()
        if self.global_iteration % self.log_save_interval == 0 and self.is_main:
            print("Iter = ", self.global_iteration, "save training data and average sampling time!")
            add_scalars(alg_tb_dict, self.writer, step=self.global_iteration)
            add_scalars(self.sampler_tb_dict.pop(), self.writer, step=self.global_iteration)
        if self.global_iteration % self.apprfunc_save_interval == 0 and self.is_main:
            self.save_apprfunc()
        if self.evaluator is not None and self.global_iteration % self.eval_interval == 0 and self.global_iteration > 0:
            self._evaluate()

    def _evaluate(self):
        with ModuleOnDevice(self.networks, getattr(self.evaluator, "device", self.sample_device)):
            ret_mean, ret_std, cost_mean, cost_std = self.evaluator.run_evaluation(self.global_iteration)
        if not self.is_main:
            return
        it = self.global_iteration
        apf = os.path.join(self.save_folder, "apprfunc")
        if ret_mean >= self.best_tar and it >= self.max_iteration / 5:
            self.best_tar = ret_mean
            print("Eval_Iter: {}, Highest total average return = {}! Current total average cost = {}".format(
                it, self.best_tar, cost_mean))
            for fn in os.listdir(apf):
                if fn.endswith("_opt.pkl"):
                    os.remove(os.path.join(apf, fn))
            torch.save(self.networks.state_dict(), os.path.join(apf, "apprfunc_{}_opt.pkl".format(it)))
        now = int(time.time() - self.start_time)
        self.writer.add_scalar(tb_tags["TRM of RL iteration"], ret_mean, it)
        self.writer.add_scalar(tb_tags["TRS of RL iteration"], ret_std, it)
        self.writer.add_scalar(tb_tags["TRM of total time"], ret_mean, now)
        self.writer.add_scalar(tb_tags["TCM of RL iteration"], cost_mean, it)
        self.writer.add_scalar(tb_tags["TCS of RL iteration"], cost_std, it)
        self.writer.add_scalar(tb_tags["TCM of total time"], cost_mean, now)

    def close(self):
        """Release the device resources of the pipeline's parts now (sampler graph + env handle,
        the algorithm's captured update graphs, the evaluator's envs), deterministically instead
        of whenever their owners are garbage collected. Idempotent."""
        fin = getattr(self, "finish_pending", None)
        if fin is not None:
            fin()
        for part in (self.sampler, self.alg, self.evaluator):
            close = getattr(part, "close", None)
            if close is not None:
                close()

    def train(self):
        while self.global_iteration < self.max_iteration:
            self.step()
        if self.is_main:
            self.save_apprfunc()
        self.writer.flush()

    def save_apprfunc(self):
        torch.save(self.networks.state_dict(),
                   os.path.join(self.save_folder, "apprfunc", "apprfunc_{}.pkl".format(self.global_iteration)))
