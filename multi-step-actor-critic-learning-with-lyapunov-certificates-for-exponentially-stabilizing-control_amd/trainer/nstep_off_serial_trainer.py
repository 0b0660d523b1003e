"""n-step off-policy serial trainer (RL/trainer/nstep_off_serial_trainer.py:22-163).

Same loop: warm-up fill, then per iteration sample -> add_batch -> sample_batch ->
model_update -> log / save / evaluate. Differences, all at the device boundary:
  * the reference moves every network to CPU around sampler.sample() (:78); here the sampler
    declares its device (`sampler.device`) and the networks stay on it;
  * replay batches are already device tensors (no `.cuda()` H2D copy, :87-89);
  * the HIP sampler is bound to the device buffer at construction so windows are emitted in
    place;
  * tensorboard is optional (in-memory writer when absent);
  * overlapped sampling (`trainer_overlap_sampling`, off by default): when the
    update of iteration k leaves the policy unchanged (k % policy_frequency != 0), the sampling of
    iteration k + 1 only depends on what precedes that update, so it is enqueued on a second stream
    right after the replay gather of iteration k and runs concurrently with the update. Same
    values as the serial order: the sampler reads only the policy (unchanged by that update) and
    writes only the window store (iteration k's batch was gathered before); the buffer bookkeeping,
    the next replay gather and every PER tree operation stay on the main stream, in order.
    Measured on one MI355X at the bench config: 567-571 M env-steps/s with it vs 578-587 M
    without (tools/overlap_ab.sh) — the persistent policy kernel takes every CU, so sharing the
    chip with the update's kernels only delays it; hence off by default.
"""
__all__ = ["NstepOffSerialTrainer"]

import os
import time
from math import inf

import torch

from ..env.hip_vector_env import drain_pending_handles
from ..utils import dist as D
from ..utils.common_utils import ModuleOnDevice
from ..utils.log_data import LogData
from ..utils.tensorboard_setup import add_scalars, make_writer, tb_tags


class NstepOffSerialTrainer:
    def __init__(self, alg, sampler, buffer, evaluator, **kwargs):
        self.alg = alg
        self.sampler = sampler
        self.buffer = buffer
        self.evaluator = evaluator
        self.per_flag = kwargs["buffer_name"] == "prioritized_replay_buffer"
        self.networks = self.alg.networks
        self.sampler.networks = self.networks
        if self.evaluator is not None:
            self.evaluator.networks = self.networks
        if kwargs.get("ini_network_dir") is not None:
            self.networks.load_state_dict(torch.load(kwargs["ini_network_dir"], weights_only=True))
        D.broadcast_module(self.networks)
        self.replay_batch_size = kwargs["replay_batch_size"]
        self.max_iteration = kwargs["max_iteration"]
        self.policy_frequency = kwargs["policy_frequency"]
        self.sample_interval = kwargs.get("sample_interval", 1)
        self.log_save_interval = kwargs["log_save_interval"]
        self.apprfunc_save_interval = kwargs["apprfunc_save_interval"]
        self.save_folder = kwargs["save_folder"]
        self.eval_interval = kwargs["eval_interval"]
        self.best_tar = -inf
        self.iteration = 0
        self.is_main = D.rank() == 0
        self.writer = make_writer(self.save_folder, flush_secs=20)
        add_scalars({tb_tags["alg_time"]: 0, tb_tags["sampler_time"]: 0}, self.writer, 0)
        self.writer.flush()
        if hasattr(self.sampler, "bind_store") and hasattr(self.buffer, "ws"):
            self.sampler.bind_store(self.buffer)
        self.sample_device = getattr(self.sampler, "device", "cpu")
        warm_calls = 0
        while self.buffer.size < kwargs["buffer_warm_size"]:
            with ModuleOnDevice(self.networks, self.sample_device):
                samples, _ = self.sampler.sample()
            self.buffer.add_batch(samples)
            warm_calls += 1
            if warm_calls > int(kwargs.get("buffer_warm_max_samples", 100000)):
                raise RuntimeError("buffer warm-up did not reach buffer_warm_size: episodes never reach n_step")
        self.sampler_tb_dict = LogData()
        self.use_gpu = kwargs.get("use_gpu", torch.cuda.is_available())
        dev = torch.device(self.sample_device)
        self.overlap = (bool(kwargs.get("trainer_overlap_sampling", False)) and dev.type == "cuda"
                        and hasattr(self.sampler, "bind_store"))
        self._side = None
        self._pending = None
        # one graph per iteration kind holding the sampling AND the update (_graph_step)
        self.graph_step = bool(kwargs.get("trainer_graph_step", os.environ.get("MSACL_GRAPH_STEP", "1") != "0"))
        self._step_graphs = {}
        self._packed_state = None  # (sampler key, policy updates, policy version) at the last graphed pack
        self.start_time = time.time()

    def _sample(self):
        with ModuleOnDevice(self.networks, self.sample_device):
            return self.sampler.sample()

    def _replay_batch(self):
        """buffer.sample_batch (:87-89); gathered straight into the update graph's static inputs
        when the algorithm replays graphs and the buffer takes an `out` (no copy before the replay)."""
        out = self.alg.replay_inputs(self.replay_batch_size) if hasattr(self.alg, "replay_inputs") else None
        if out is not None:
            return self.buffer.sample_batch(self.replay_batch_size, out=out)
        if getattr(self.alg, "wants_joint_batch", False) and hasattr(self.buffer, "_joint_shapes"):
            return self.buffer.sample_batch(self.replay_batch_size, joint=True)
        return self.buffer.sample_batch(self.replay_batch_size)

    def _drawn_update(self):
        """The replay draw runs inside the algorithm's replayed update (the buffer's one-launch
        draw + gather captured as the graph's first node): graph replay under way, a plain
        device buffer (its draw counter on the device), no PER, no overlapped sampling (that
        orders the next sampling after an eager gather)."""
        return (not self.per_flag and not self._overlap_next() and getattr(self.buffer, "graph_draw", False)
                and hasattr(self.alg, "model_update_drawn")
                and self.alg.replay_inputs(self.replay_batch_size) is not None)

    def _update(self, replay_samples):
        """alg.model_update on the drawn batch, or with the draw inside the replay (None)."""
        if replay_samples is None:
            B, buf = self.replay_batch_size, self.buffer
            return self.alg.model_update_drawn(lambda out: buf.sample_batch(B, out=out), self.iteration)
        return self.alg.model_update(replay_samples, self.iteration)

    def replay_and_update(self):
        """The replay draw and the update of one step (step()'s middle part, for measurements)."""
        rs = None if self._drawn_update() else self._replay_batch()
        return self._update(rs)

    def _overlap_next(self):
        """Sampling of iteration + 1 may run beside this iteration's update."""
        return (self.overlap and self.iteration % self.policy_frequency != 0
                and (self.iteration + 1) % self.sample_interval == 0 and self.iteration + 1 <= self.max_iteration)

    def _graph_step(self):
        """The iteration's sampling and update replayed as ONE HIP graph instead of two (the
        sampler's and the update's): the graph-to-graph transition between them (~9 us on the
        device) becomes a kernel boundary inside the graph. Applies once both parts were run
        eagerly (sampler: its first horizon; update: each branch's first call) to the plain
        drawn-update path (sampling every iteration, no PER, no overlapped sampling, sampler time
        not synchronised). The captured work is exactly the two graphs' in their order.
        -> (True, model_update's return value), or None to take the separate calls."""
        if (not self.graph_step or self.sample_interval != 1 or self._pending is not None or self.per_flag
                or not self._drawn_update() or getattr(self.sampler, "device", None) != getattr(self.alg, "device", None)):
            return None
        sparts, aparts = getattr(self.sampler, "step_graph_parts", None), getattr(self.alg, "drawn_step_parts", None)
        if sparts is None or aparts is None:
            return None
        sp = sparts()
        if sp is None:
            return None
        B, buf = self.replay_batch_size, self.buffer
        ap = aparts(lambda out: buf.sample_batch(B, out=out), self.iteration)
        if ap is None:
            return None
        # the policy pack (two launches, ~11 us) only when the parameters may have changed since the
        # last graphed pack: a policy update since (the algorithm's host count, every update path)
        # or any in-place write through torch (the parameters' version counters)
        skey = sp[0]
        pv = getattr(self.alg, "policy_updates", None)
        vfn = getattr(self.sampler, "policy_version", None)
        state = (skey, pv, vfn() if vfn is not None else None)
        pack = not (pv is not None and vfn is not None and self._packed_state == state)
        if not pack:
            sp = sparts(pack=False)
        skey, pre, sbody, spost = sp
        akey, abody, apost = ap
        key = (skey, akey, pack)
        if pack:
            self._packed_state = state
        pre()
        t0, start = time.perf_counter(), time.time()
        ent = self._step_graphs.get(key)
        if ent is None:
            # graphs of an older sampler key (other policy / observation buffers) or of older static
            # update inputs (the algorithm rebuilt them: akey[2:] is their generation) are dead
            self._step_graphs = {k: v for k, v in self._step_graphs.items() if k[0] == skey and k[1][2:] == akey[2:]}
            g = torch.cuda.CUDAGraph()
            with D.cuda_graph(g):
                sbody()
                outs = abody()
            drain_pending_handles()  # env handles released by a finaliser during the capture
            ent = self._step_graphs[key] = (g, outs)
        g, outs = ent
        self.networks.train()
        g.replay()  # (a policy update inside advances alg.policy_updates in apost: the next step packs)
        samples, stb = spost(t0)
        self.buffer.add_batch(samples)
        self.sampler_tb_dict.add_average(stb)
        return True, apost(outs, start)

    def step(self):
        graphed = self._graph_step()
        if graphed is not None:
            alg_tb_dict = graphed[1]
            if (self.iteration % self.policy_frequency == 0 and self.iteration % self.log_save_interval == 0
                    and self.is_main):
                print("Iter = ", self.iteration, "save training data!")
                add_scalars(alg_tb_dict, self.writer, step=self.iteration)
            self._step_tail()
            return
        if self.iteration % self.sample_interval == 0:
            if self._pending is not None:  # enqueued on the side stream during the last update
                sampler_samples, sampler_tb_dict = self._pending
                self._pending = None
                torch.cuda.current_stream(self._side.device).wait_stream(self._side)
            else:
                sampler_samples, sampler_tb_dict = self._sample()
            self.buffer.add_batch(sampler_samples)
            self.sampler_tb_dict.add_average(sampler_tb_dict)
        replay_samples = None if self._drawn_update() else self._replay_batch()
        if self._overlap_next():
            if self._side is None:
                self._side = torch.cuda.Stream(device=torch.device(self.sample_device))
            main = torch.cuda.current_stream(self._side.device)
            self._side.wait_stream(main)  # after the replay gather above
            with torch.cuda.stream(self._side):
                self._pending = self._sample()
        self.networks.train()
        if self.per_flag:
            alg_tb_dict, idx, new_priority = self.alg.model_update(replay_samples, self.iteration)
            self.buffer.update_batch(idx, new_priority)
            if alg_tb_dict is not None and self.iteration % self.log_save_interval == 0 and self.is_main:
                add_scalars(alg_tb_dict, self.writer, step=self.iteration)
        elif self.iteration % self.policy_frequency == 0:
            alg_tb_dict = self._update(replay_samples)
            if self.iteration % self.log_save_interval == 0 and self.is_main:
                print("Iter = ", self.iteration, "save training data!")
                add_scalars(alg_tb_dict, self.writer, step=self.iteration)
        else:
            self._update(replay_samples)
        self._step_tail()

    def _step_tail(self):
        self.networks.eval()
        if self.iteration % self.log_save_interval == 0:
            check = getattr(self.sampler, "check_errors", None)  # device sampler health (every rank)
            if check is not None:
                check()
        if self.iteration % self.log_save_interval == 0 and self.is_main:
            print("Iter = ", self.iteration, "save average sampling time!")
            add_scalars(self.sampler_tb_dict.pop(), self.writer, step=self.iteration)
        if self.iteration % self.apprfunc_save_interval == 0 and self.is_main:
            self.save_apprfunc()
        if self.evaluator is not None and self.iteration % self.eval_interval == 0 and self.iteration > 0:
            self._evaluate()

    def _evaluate(self):
        with ModuleOnDevice(self.networks, getattr(self.evaluator, "device", self.sample_device)):
            ret_mean, ret_std, cost_mean, cost_std = self.evaluator.run_evaluation(self.iteration)
        if not self.is_main:
            return
        apf = os.path.join(self.save_folder, "apprfunc")
        if ret_mean >= self.best_tar and self.iteration >= self.max_iteration / 5:
            self.best_tar = ret_mean
            print("Eval_Iter: {}, Highest total average return = {}! Current total average cost = {}".format(
                self.iteration, self.best_tar, cost_mean))
            for fn in os.listdir(apf):
                if fn.endswith("_opt.pkl"):
                    os.remove(os.path.join(apf, fn))
            torch.save(self.networks.state_dict(), os.path.join(apf, "apprfunc_{}_opt.pkl".format(self.iteration)))
        self.writer.add_scalar(tb_tags["Buffer RAM of RL iteration"], self.buffer.__get_RAM__(), self.iteration)
        self.writer.add_scalar(tb_tags["TRM of RL iteration"], ret_mean, self.iteration)
        self.writer.add_scalar(tb_tags["TRS of RL iteration"], ret_std, self.iteration)
        self.writer.add_scalar(tb_tags["TRM of total time"], ret_mean, int(time.time() - self.start_time))
        self.writer.add_scalar(tb_tags["TCM of RL iteration"], cost_mean, self.iteration)
        self.writer.add_scalar(tb_tags["TCS of RL iteration"], cost_std, self.iteration)
        self.writer.add_scalar(tb_tags["TCM of total time"], cost_mean, int(time.time() - self.start_time))

    def finish_pending(self):
        """Join an overlapped sampling still in flight (its windows join the buffer)."""
        if self._pending is not None:
            samples, tb = self._pending
            self._pending = None
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
            self.buffer.add_batch(samples)
            self.sampler_tb_dict.add_average(tb)

    def close(self):
        """Release the device resources of the pipeline's parts now (sampler graph + env handle,
        the algorithm's captured update graphs, the evaluator's envs), deterministically instead
        of whenever their owners are garbage collected. Idempotent."""
        fin = getattr(self, "finish_pending", None)
        if fin is not None:
            fin()
        self._step_graphs = {}  # (their captured work references the parts' device buffers)
        for part in (self.sampler, self.alg, self.evaluator):
            close = getattr(part, "close", None)
            if close is not None:
                close()

    def train(self):
        while self.iteration <= self.max_iteration:
            self.step()
            self.iteration += 1
        self.finish_pending()
        if self.is_main:
            self.save_apprfunc()
        self.writer.flush()

    def save_apprfunc(self):
        torch.save(self.networks.state_dict(),
                   os.path.join(self.save_folder, "apprfunc", "apprfunc_{}.pkl".format(self.iteration)))
