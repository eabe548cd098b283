"""`cxxnet <conf> [key=value ...]` -- the task driver.

Behavioural parity with reference src/cxxnet_main.cpp (CXXNetLearnTask):
  tasks train / finetune / pred / extract; model naming model_dir/%04d.model;
  `continue=1` resumes from the latest model file; `model_in` infers start_counter from
  the file name; 0000.model is written before training; eval lines go to stderr as
  "[round]\\ttrain-error:x\\ttest-error:y"; progress to stdout every print_step batches;
  `test_io=1` runs only the data pipeline; a value of `default` is ignored.
Multi-GPU: `dev=gpu:0-7` (or gpu:0,1,...) launches one process per listed GPU through
torch.distributed.run (RCCL over xGMI) with this same command line.
"""
from __future__ import annotations

import os
import struct
import subprocess
import sys
import time
from typing import List, Optional, Tuple

import numpy as np


class LearnTask:
    def __init__(self):
        self.net_type = 0
        self.reset_net_type = -1
        self.print_step = 100
        self.continue_training = 0
        self.save_period = 1
        self.start_counter = 0
        self.name_model_in = "NULL"
        self.name_model_dir = "models"
        self.num_round = 10
        self.max_round = 2 ** 31 - 1
        self.silent = 0
        self.task = "train"
        self.device = "gpu"
        self.test_io = 0
        self.extract_node_name = ""
        self.output_format = 1
        self.name_pred = "pred.txt"
        self.cfg: List[Tuple[str, str]] = []
        self.trainer = None
        self.itr_train = None
        self.itr_pred = None
        self.itr_evals = []
        self.eval_names = []
        # checkpoint sidecar with momentum / second moment (<model>.state), restored on continue
        self.save_opt_state = 0
        # failure detection: abort the process if one update takes longer than this (seconds)
        self.step_timeout = 0.0
        self._last_progress = 0.0

    # ------------------------------------------------------------------ config
    def set_param(self, name: str, val: str):
        if val == "default":
            return
        if name == "net_type":
            self.net_type = int(val)
        elif name == "reset_net_type":
            self.reset_net_type = int(val)
        elif name == "print_step":
            self.print_step = int(val)
        elif name == "continue":
            self.continue_training = int(val)
        elif name == "save_model":
            self.save_period = int(val)
        elif name == "start_counter":
            self.start_counter = int(val)
        elif name == "model_in":
            self.name_model_in = val
        elif name == "model_dir":
            self.name_model_dir = val
        elif name == "num_round":
            self.num_round = int(val)
        elif name == "max_round":
            self.max_round = int(val)
        elif name == "silent":
            self.silent = int(val)
        elif name == "task":
            self.task = val
        elif name == "dev":
            self.device = val
        elif name == "test_io":
            self.test_io = int(val)
        elif name == "extract_node_name":
            self.extract_node_name = val
        elif name == "output_format":
            self.output_format = 1 if val == "txt" else 0
        elif name == "save_optimizer_state":
            self.save_opt_state = int(val)
        elif name == "step_timeout":
            self.step_timeout = float(val)
        self.cfg.append((name, val))

    @property
    def rank(self):
        from .parallel import world_info
        return world_info()[0]

    def log(self, *a, **k):
        if not self.silent and self.rank == 0:
            print(*a, **k)
            sys.stdout.flush()

    def run(self, argv: List[str]) -> int:
        if len(argv) < 1:
            print("Usage: <config> [key=value ...]")
            return 0
        from . import native
        for k, v in native.rt().parse_config_file(argv[0]):
            self.set_param(k, v)
        for a in argv[1:]:
            if "=" in a:
                k, v = a.split("=", 1)
                self.set_param(k, v)
        from .parallel import init_distributed
        init_distributed()
        self.init()
        self.log("initializing end, start working")
        if self.task in ("train", "finetune"):
            self.task_train()
        elif self.task in ("pred", "pred_raw"):
            self.task_predict()
        elif self.task in ("extract", "extract_feature"):
            self.task_extract()
        return 0

    # ------------------------------------------------------------------ init
    def _create_net(self):
        from .nnet import create_net
        if self.reset_net_type != -1:
            self.net_type = self.reset_net_type
        tr = create_net(self.net_type)
        for k, v in self.cfg:
            tr.set_param(k, v)
        return tr

    def _model_path(self, counter: int) -> str:
        return os.path.join(self.name_model_dir, "%04d.model" % counter)

    def sync_latest_model(self) -> bool:
        s = self.start_counter
        last = None
        while os.path.exists(self._model_path(s)):
            last = self._model_path(s)
            s += 1
        if last is None:
            return False
        with open(last, "rb") as f:
            data = f.read()
        self.net_type = struct.unpack_from("<i", data, 0)[0]
        self.trainer = self._create_net()
        self.trainer.load_model(data, 4)
        self._load_state_sidecar(last)
        self.start_counter = s - 1
        return True

    def _load_state_sidecar(self, model_path: str):
        if self.save_opt_state and os.path.exists(model_path + ".state"):
            self.trainer.load_optimizer_state(model_path + ".state")
            self.log(f"restored optimizer state from {model_path}.state")

    def load_model(self):
        base = os.path.basename(self.name_model_in)
        try:
            self.start_counter = int(base.split(".")[0])
        except ValueError:
            print("WARNING: Cannot infer start_counter from model name. Specify it in config if needed")
        with open(self.name_model_in, "rb") as f:
            data = f.read()
        self.net_type = struct.unpack_from("<i", data, 0)[0]
        self.trainer = self._create_net()
        self.trainer.load_model(data, 4)
        self._load_state_sidecar(self.name_model_in)
        self.start_counter += 1

    def copy_model(self):
        with open(self.name_model_in, "rb") as f:
            data = f.read()
        self.net_type = struct.unpack_from("<i", data, 0)[0]
        self.trainer = self._create_net()
        self.trainer.init_model()
        self.trainer.copy_model_from_bytes(data, 4)

    def save_model(self):
        path = self._model_path(self.start_counter)
        self.start_counter += 1
        if self.save_period == 0 or self.start_counter % self.save_period != 0:
            return
        # collective on EVERY rank (sharded data parallelism gathers the fp32 masters and the
        # optimizer state here); rank 0 then writes without entering another collective
        self.trainer.prepare_save(opt_state=bool(self.save_opt_state))
        if self.rank != 0:
            return
        os.makedirs(self.name_model_dir, exist_ok=True)
        blob = self.trainer.save_model(sync=False)
        with open(path + ".tmp", "wb") as f:
            f.write(struct.pack("<i", self.net_type))
            f.write(blob)
        os.replace(path + ".tmp", path)
        if self.save_opt_state:
            self.trainer.save_optimizer_state(path + ".state.tmp", sync=False)
            os.replace(path + ".state.tmp", path + ".state")

    def init(self):
        if self.task == "train" and self.continue_training:
            if not self.sync_latest_model():
                raise RuntimeError("Init: Cannot find models for continue training. "
                                   "Please specify it by model_in instead.")
            print(f"Init: Continue training from round {self.start_counter}")
            self.create_iterators()
            return
        self.continue_training = 0
        if self.name_model_in == "NULL":
            if self.task != "train":
                raise RuntimeError("must specify model_in if not training")
            self.trainer = self._create_net()
            self.trainer.init_model()
        elif self.task == "finetune":
            self.copy_model()
        else:
            self.load_model()
        self.create_iterators()

    def create_iterators(self):
        from .io import create_iterator
        flag = 0
        evname = ""
        itcfg: List[Tuple[str, str]] = []
        defcfg: List[Tuple[str, str]] = []
        for name, val in self.cfg:
            if name == "data":
                flag = 1
                continue
            if name == "eval":
                evname = val
                flag = 2
                continue
            if name == "pred":
                flag = 3
                self.name_pred = val
                continue
            if name == "iter" and val == "end":
                if flag == 0:
                    raise RuntimeError("wrong configuration file")
                if flag == 1 and self.task not in ("pred", "pred_raw"):
                    if self.itr_train is not None:
                        raise RuntimeError("can only have one data")
                    self.itr_train = create_iterator(itcfg)
                if flag == 2 and self.task not in ("pred", "pred_raw"):
                    self.itr_evals.append(create_iterator(itcfg))
                    self.eval_names.append(evname)
                if flag == 3 and self.task in ("pred", "pred_raw", "extract", "extract_feature"):
                    if self.itr_pred is not None:
                        raise RuntimeError("can only have one data:test")
                    self.itr_pred = create_iterator(itcfg)
                flag = 0
                itcfg = []
                continue
            if flag == 0:
                defcfg.append((name, val))
            else:
                itcfg.append((name, val))
        for it in [self.itr_train, self.itr_pred] + self.itr_evals:
            if it is not None:
                for k, v in defcfg:
                    it.set_param(k, v)
                it.init()

    # ------------------------------------------------------------------ tasks
    def task_predict(self):
        if self.itr_pred is None:
            raise RuntimeError("must specify a predict iterator to generate predictions")
        self.log("start predicting...")
        raw = self.task == "pred_raw"
        out = []
        self.itr_pred.before_first()
        while self.itr_pred.next():
            b = self.itr_pred.value()
            if raw:  # whole output row per instance (used by the Kaggle bowl submission)
                top = len(self.trainer.net.nodes) - 1
                pred = self.trainer.forward_to([top], b)[0].reshape(b.batch_size, -1)
            else:
                pred = self.trainer.predict(b)
            sz = len(pred) - b.num_batch_padd
            out.extend(pred[:sz].tolist())
        if self.rank == 0:
            with open(self.name_pred, "w") as f:
                for v in out:
                    if raw:
                        f.write("".join("%g " % x for x in v) + "\n")
                    else:
                        f.write("%g\n" % v)
        self.log(f"finished prediction, write into {self.name_pred}")

    def task_extract(self):
        if self.itr_pred is None:
            raise RuntimeError("must specify a predict iterator to generate predictions")
        if not self.extract_node_name:
            raise RuntimeError("extract node name must be specified in task extract_feature.")
        self.log("start predicting...")
        nrow = 0
        dshape = (0, 0, 0)
        fo = open(self.name_pred, "w" if self.output_format else "wb") if self.rank == 0 else None
        self.itr_pred.before_first()
        while self.itr_pred.next():
            b = self.itr_pred.value()
            feat = self.trainer.extract_feature(b, self.extract_node_name)
            sz = feat.shape[0] - b.num_batch_padd
            nrow += sz
            if sz:
                dshape = tuple(feat.shape[1:]) if feat.ndim == 4 else (1, 1, int(np.prod(feat.shape[1:])))
            if fo is not None:
                rows = feat[:sz].reshape(sz, -1).astype(np.float32)
                if self.output_format:
                    for r in rows:
                        fo.write("".join("%g " % v for v in r) + "\n")
                else:
                    fo.write(rows.tobytes())
        if fo is not None:
            fo.close()
            with open(self.name_pred + ".meta", "w") as fm:
                fm.write("%d,%d,%d,%d\n" % (nrow, dshape[0], dshape[1], dshape[2]))
        self.log(f"finished prediction, write into {self.name_pred}")

    def _eval_line(self, r: Optional[int]) -> str:
        s = "" if r is None else f"[{r}]"
        if not self.itr_evals:
            s += self.trainer.evaluate(None, "train")
        for it, name in zip(self.itr_evals, self.eval_names):
            s += self.trainer.evaluate(it, name)
        return s

    def task_train(self):
        start = time.time()
        elapsed = 0
        if self.continue_training == 0 and self.name_model_in == "NULL":
            self.save_model()
        else:
            self.log(f"continuing from round {self.start_counter - 1}", end="")
            line = ""
            for it, name in zip(self.itr_evals, self.eval_names):
                line += self.trainer.evaluate(it, name)
            if self.rank == 0:
                sys.stderr.write(line + "\n")
                sys.stderr.flush()
        if self.itr_train is None:
            return
        if self.test_io:
            self.log("start I/O test")
        self._start_watchdog()
        cc = self.max_round
        while self.start_counter <= self.num_round and cc > 0:
            cc -= 1
            self.log(f"update round {self.start_counter - 1}", end="")
            sample_counter = 0
            self.trainer.start_round(self.start_counter)
            self.itr_train.before_first()
            t_mark, n_mark = time.perf_counter(), 0
            while self.itr_train.next():
                if not self.test_io:
                    self.trainer.update(self.itr_train.value())
                self._last_progress = time.time()
                sample_counter += 1
                if sample_counter % self.print_step == 0:
                    elapsed = int(time.time() - start)
                    self.log("\r" + " " * 63 + "\r" +
                             f"round {self.start_counter - 1:8d}:[{sample_counter:8d}] {elapsed} sec elapsed", end="")
                    if getattr(self.trainer, "profile_step", 0):
                        # wall clock over the last print_step updates (the host runs at most a
                        # few steps ahead of the GPU, so this is the training rate) + HIP-event
                        # split of the GPU step
                        now = time.perf_counter()
                        ips = (sample_counter - n_mark) * self.trainer.batch_size / max(now - t_mark, 1e-9)
                        t_mark, n_mark = now, sample_counter
                        self.log(f"\nwall {ips:.0f} img/s; " + self.trainer.timing_report(), end="")
            if not self.test_io:
                line = self._eval_line(self.start_counter)
                if self.rank == 0:
                    sys.stderr.write(line + "\n")
                    sys.stderr.flush()
            elapsed = int(time.time() - start)
            self.save_model()
            self._last_progress = time.time()  # evaluation / checkpointing is progress too
        self.log(f"\nupdating end, {elapsed} sec in all")


    def _start_watchdog(self):
        """step_timeout > 0: a daemon thread ends the process (exit code 3) when no update
        finished for that long -- a hung collective or kernel fails fast instead of holding
        every rank of the job."""
        if self.step_timeout <= 0:
            return
        import threading
        self._last_progress = time.time()

        def watch():
            while True:
                time.sleep(min(1.0, self.step_timeout / 4))
                if time.time() - self._last_progress > self.step_timeout:
                    sys.stderr.write(f"step_timeout: no update finished in {self.step_timeout:g} s "
                                     f"(rank {self.rank}); aborting\n")
                    sys.stderr.flush()
                    os._exit(3)

        threading.Thread(target=watch, daemon=True, name="cxxnet-watchdog").start()


def _maybe_spawn_ranks(argv: List[str]) -> Optional[int]:
    """dev=gpu:a-b / gpu:a,b,... with several GPUs and not already under torchrun:
    re-launch this command as one process per GPU (child process; we exit with its code)."""
    if "WORLD_SIZE" in os.environ:
        return None
    dev = None
    batch = None
    try:
        from . import native
        for k, v in native.rt().parse_config_file(argv[0]):
            if k == "dev":
                dev = v
            elif k == "batch_size":
                batch = int(v)
    except Exception:
        return None
    for a in argv[1:]:
        if a.startswith("dev="):
            dev = a.split("=", 1)[1]
        elif a.startswith("batch_size="):
            batch = int(a.split("=", 1)[1])
    if not dev or not dev.startswith("gpu") or ":" not in dev:
        return None
    from .nnet.trainer import parse_devices, prune_devices
    _, ids = parse_devices(dev)
    if batch is not None and len(ids) > 1:
        # the reference drops the devices a batch cannot cover (nnet_impl-inl.hpp:344-354)
        n = prune_devices(batch, len(ids))
        if n < len(ids):
            step = max((batch + len(ids) - 1) // len(ids), 1)
            print(f"Warning: The number of devices is induce mini-batch={step}\n"
                  f"We can equally use {n} devices to cover the batch_size")
            ids = ids[:n]
    if len(ids) <= 1:  # one device (possibly after pruning): this process runs on device ids[0]
        return None
    env = dict(os.environ)
    env["HIP_VISIBLE_DEVICES"] = ",".join(str(i) for i in ids)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    port = env.get("CXXNET_MASTER_PORT")
    if not port:  # a free local port: a fixed default collides with any other job on the host
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = str(s.getsockname()[1])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={len(ids)}",
           "--master-addr", "127.0.0.1", "--master-port", port,
           "-m", "cxxnet_amd"] + argv
    return subprocess.call(cmd, env=env)


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    rc = _maybe_spawn_ranks(argv) if argv else None
    if rc is not None:
        return rc
    return LearnTask().run(argv)


if __name__ == "__main__":
    sys.exit(main())
