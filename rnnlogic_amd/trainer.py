"""TrainerPredictor, API-compatible with the reference's src/trainer.py:10-289
(train / compute_H / evaluate / load / save).

Same data flow as the reference — DistributedSampler(world, rank) over the
per-relation batches (its padding duplicates included), label smoothing, the
softmax cross-entropy over the mask, DDP with find_unused_parameters, comm.cat
of the rank lists, the tie-expectation metrics over unique (h, r, t) divided by
the padded count — with two differences in *how*, not *what*:
  * evaluate() scores all of the rank's rows in one PredictorPlus.forward_rows
    launch (rows are independent in eval mode) and computes the filtered ranks
    on the device, instead of one forward and a Python loop per row;
  * training forwards run PredictorPlus's differentiable path (HIP grounding,
    autograd on the exported path-count COO).
"""
import logging
import os
from itertools import islice

import torch
from torch import distributed as dist
from torch import nn
from torch.utils import data as torch_data

from . import comm
from .data import DeviceTrainBatches


class _SizedIter(object):
    """len() + iteration over fn(index) for the sampler's indices."""

    def __init__(self, sampler, fn):
        self.sampler, self.fn = sampler, fn

    def __len__(self):
        return len(self.sampler)

    def __iter__(self):
        return (self.fn(i) for i in self.sampler)


class TrainerPredictor(object):

    def __init__(self, model, train_set, valid_set, test_set, optimizer, scheduler=None, gpus=None, num_worker=0):
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        self.gpus = gpus
        self.num_worker = num_worker
        if gpus is None:
            self.device = torch.device("cpu")
        else:
            if len(gpus) != self.world_size:
                error_msg = "World size is %d but found %d GPUs in the argument"
                if self.world_size == 1:
                    error_msg += ". Did you launch with `python -m torch.distributed.launch`?"
                raise ValueError(error_msg % (self.world_size, len(gpus)))
            self.device = torch.device(gpus[self.rank % len(gpus)])
        if self.world_size > 1 and not dist.is_initialized():
            if self.rank == 0:
                logging.info("Initializing distributed process group")
            backend = "gloo" if gpus is None else "nccl"
            comm.init_process_group(backend, init_method="env://")
        if self.rank == 0:
            logging.info("Preprocess training set")
        if self.world_size > 1:
            model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
        if self.device.type == "cuda":
            model = model.cuda(self.device)
        self.model = model
        self.train_set = train_set
        self.valid_set = valid_set
        self.test_set = test_set
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.device_batches = True  # GPU: training batches built on the device (f3)

    # ------------------------------------------------------------------ train
    def _loader(self, dataset):
        """(sampler, iterable of batches).  On a GPU the training batches are
        built on the device (data.DeviceTrainBatches, same tensors as
        TrainDataset.__getitem__) in the sampler's order; otherwise the
        reference's DataLoader."""
        sampler = torch_data.DistributedSampler(dataset, self.world_size, self.rank)
        if self.device.type == "cuda" and dataset is self.train_set and self.device_batches:
            if getattr(self, "_dev_batches", None) is None:
                self._dev_batches = DeviceTrainBatches(self.train_set, self.device)
            dev = self._dev_batches
            return sampler, _SizedIter(sampler, lambda i: [x.unsqueeze(0) for x in dev[i]])
        return sampler, torch_data.DataLoader(dataset, 1, sampler=sampler, num_workers=self.num_worker)

    def train(self, batch_per_epoch, smoothing, print_every):
        """trainer.py:48-105."""
        if comm.get_rank() == 0:
            logging.info(">>>>> Predictor: Training")
        self.train_set.make_batches()
        sampler, dataloader = self._loader(self.train_set)
        batch_per_epoch = batch_per_epoch or len(dataloader)
        model = self.model
        if self.world_size > 1:
            if self.device.type == "cuda":
                model = nn.parallel.DistributedDataParallel(model, device_ids=[self.device],
                                                            find_unused_parameters=True)
            else:
                model = nn.parallel.DistributedDataParallel(model, find_unused_parameters=True)
        model.train()
        total_loss, total_size = 0.0, 0.0
        sampler.set_epoch(0)
        for batch_id, batch in enumerate(islice(dataloader, batch_per_epoch)):
            loss, size = self.train_step(model, batch, smoothing)
            if loss is not None:
                total_loss += loss
                total_size += size
            if (batch_id + 1) % print_every == 0:
                if comm.get_rank() == 0:
                    logging.info("{} {} {:.6f} {:.1f}".format(batch_id + 1, len(dataloader), total_loss / print_every,
                                                             total_size / print_every))
                total_loss, total_size = 0.0, 0.0
        if self.scheduler:
            self.scheduler.step()

    def train_step(self, model, batch, smoothing):
        """One optimizer step on one batch (trainer.py:72-98); returns
        (loss, mask size) or (None, None) when the batch has no candidate."""
        all_h, all_r, all_t, target, edges_to_remove = [x.squeeze(0) for x in batch]
        target_t = torch.nn.functional.one_hot(all_t, self.train_set.graph.entity_size)
        if self.device.type == "cuda":
            all_h = all_h.cuda(device=self.device)
            all_r = all_r.cuda(device=self.device)
            target = target.cuda(device=self.device)
            edges_to_remove = edges_to_remove.cuda(device=self.device)
            target_t = target_t.cuda(device=self.device)
        target = target * smoothing + target_t * (1 - smoothing)
        logits, mask = model(all_h, all_r, edges_to_remove)
        if mask.sum().item() == 0:
            return None, None
        logits = (torch.softmax(logits, dim=1) + 1e-8).log()
        loss = -(logits[mask] * target[mask]).sum() / torch.clamp(target[mask].sum(), min=1)
        loss.backward()
        self.optimizer.step()
        self.optimizer.zero_grad()
        return loss.item(), mask.sum().item()

    # ------------------------------------------------------------------ H scores
    @torch.no_grad()
    def compute_H(self, print_every):
        """trainer.py:107-143 (the model must provide compute_H, e.g. Predictor)."""
        if comm.get_rank() == 0:
            logging.info(">>>>> Predictor: Computing H scores of rules")
        _, dataloader = self._loader(self.train_set)
        model = self.model
        model.eval()
        all_H_score = torch.zeros(model.num_rules, device=self.device)
        for batch_id, batch in enumerate(dataloader):
            all_h, all_r, all_t, target, edges_to_remove = [x.squeeze(0) for x in batch]
            if self.device.type == "cuda":
                all_h = all_h.cuda(device=self.device)
                all_r = all_r.cuda(device=self.device)
                all_t = all_t.cuda(device=self.device)
                edges_to_remove = edges_to_remove.cuda(device=self.device)
            H, index = model.compute_H(all_h, all_r, all_t, edges_to_remove)
            if H is not None and index is not None:
                all_H_score[index] += H / len(model.graph.train_facts)
            if (batch_id + 1) % print_every == 0 and comm.get_rank() == 0:
                logging.info("{} {}".format(batch_id + 1, len(dataloader)))
        if self.world_size > 1:
            all_H_score = comm.stack(all_H_score).sum(0)
        return all_H_score.data.cpu().numpy().tolist()

    # ------------------------------------------------------------------ evaluate
    @staticmethod
    def filtered_ranks(logits, mask, flag, all_t, num_entities):
        """(L, H) per row, trainer.py:191-203: L = #(flagged scores > s_t) + 1,
        H = #(flagged scores >= s_t) + 2, or (1, |E| + 1) when t is not a
        candidate — computed for all rows at once on the device."""
        rows = torch.arange(all_t.numel(), device=logits.device)
        val = logits[rows, all_t].unsqueeze(1)
        L = ((logits > val) & flag).sum(1) + 1
        H = ((logits >= val) & flag).sum(1) + 2
        hit = mask[rows, all_t]
        L = torch.where(hit, L, torch.ones_like(L))
        H = torch.where(hit, H, torch.full_like(H, num_entities + 1))
        return L, H

    @staticmethod
    def rank_metrics(ranks, expectation=True):
        """trainer.py:207-238 on an (N, 5) [h, r, t, L, H] list: metrics over the
        unique (h, r, t), divided by N (the sampler's padding included)."""
        query2LH = dict()
        for h, r, t, L, H in ranks:
            query2LH[(h, r, t)] = (L, H)
        hit1, hit3, hit10, mr, mrr = 0.0, 0.0, 0.0, 0.0, 0.0
        for (L, H) in query2LH.values():
            if expectation:
                for rank in range(L, H):
                    if rank <= 1:
                        hit1 += 1.0 / (H - L)
                    if rank <= 3:
                        hit3 += 1.0 / (H - L)
                    if rank <= 10:
                        hit10 += 1.0 / (H - L)
                    mr += rank / (H - L)
                    mrr += 1.0 / rank / (H - L)
            else:
                rank = H - 1
                hit1 += rank <= 1
                hit3 += rank <= 3
                hit10 += rank <= 10
                mr += rank
                mrr += 1.0 / rank
        n = len(ranks)
        return dict(Data=len(query2LH), Hit1=hit1 / n, Hit3=hit3 / n, Hit10=hit10 / n, MR=mr / n, MRR=mrr / n)

    @torch.no_grad()
    def evaluate(self, split, expectation=True):
        """trainer.py:145-248 -> MRR."""
        if comm.get_rank() == 0:
            logging.info(">>>>> Predictor: Evaluating on {}".format(split))
        test_set = getattr(self, "%s_set" % split)
        _, dataloader = self._loader(test_set)
        model = self.model
        model.eval()
        E = test_set.graph.entity_size
        hs, rs, ts, flags = [], [], [], []
        for batch in dataloader:
            all_h, all_r, all_t, flag = [x.squeeze(0) for x in batch]
            hs.append(all_h)
            rs.append(all_r)
            ts.append(all_t)
            flags.append(flag)
        ranks = torch.zeros((0, 5), dtype=torch.long)
        if hs:
            all_h, all_r, all_t = torch.cat(hs), torch.cat(rs), torch.cat(ts)
            dev = self.device
            all_h, all_r, all_t = all_h.to(dev), all_r.to(dev), all_t.to(dev)
            if hasattr(model, "forward_rows") and dev.type == "cuda":
                logits, mask = model.forward_rows(all_h, all_r, None)
            else:  # per batch, as the reference (e.g. Predictor)
                out = [model(h.to(dev), r.to(dev), None) for h, r in zip(hs, rs)]
                logits, mask = torch.cat([o[0] for o in out]), torch.cat([o[1] for o in out])
            flag = torch.cat(flags).to(dev)
            L, H = self.filtered_ranks(logits, mask, flag, all_t, E)
            ranks = torch.stack([all_h, all_r, all_t, L, H], 1).to(torch.long)
        if self.world_size > 1:
            ranks = comm.cat(ranks.to(self.device))
        m = self.rank_metrics(ranks.cpu().numpy().tolist(), expectation)
        if comm.get_rank() == 0:
            logging.info("Data : {}".format(m["Data"]))
            logging.info("Hit1 : {:.6f}".format(m["Hit1"]))
            logging.info("Hit3 : {:.6f}".format(m["Hit3"]))
            logging.info("Hit10: {:.6f}".format(m["Hit10"]))
            logging.info("MR   : {:.6f}".format(m["MR"]))
            logging.info("MRR  : {:.6f}".format(m["MRR"]))
        return m["MRR"]

    # ------------------------------------------------------------------ checkpoints
    def load(self, checkpoint, load_optimizer=True):
        """trainer.py:250-271."""
        if comm.get_rank() == 0:
            logging.info("Load checkpoint from %s" % checkpoint)
        state = torch.load(os.path.expanduser(checkpoint), map_location=self.device, weights_only=True)
        self.model.load_state_dict(state["model"])
        if load_optimizer:
            self.optimizer.load_state_dict(state["optimizer"])
            for st in self.optimizer.state.values():
                for k, v in st.items():
                    if isinstance(v, torch.Tensor):
                        st[k] = v.to(self.device)
        comm.synchronize()

    def save(self, checkpoint):
        """trainer.py:273-289."""
        if comm.get_rank() == 0:
            logging.info("Save checkpoint to %s" % checkpoint)
        if self.rank == 0:
            torch.save({"model": self.model.state_dict(), "optimizer": self.optimizer.state_dict()},
                       os.path.expanduser(checkpoint))
        comm.synchronize()
