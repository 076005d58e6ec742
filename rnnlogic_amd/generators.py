"""The EM loop's rule generator, API-compatible with the reference's
src/generators.py:3-37.

An LSTM over rule sequences [head, body..., END] whose input at every step is
the token embedding concatenated with the head relation's embedding; a linear
head predicts the next token over the |R| relations + END.  The module tree
(`embedding`, `rnn`, `linear`) and its construction order are the reference's,
so state_dict keys/shapes match and a seeded construction draws the same
initial weights.  This is plain PyTorch-ROCm (SURVEY §8 north_star: the
generator stays in PyTorch); the EM trainer around it is
trainer.TrainerGenerator.
"""
import torch
import torch.nn.functional as F


class Generator(torch.nn.Module):

    def __init__(self, graph, num_layers, embedding_dim, hidden_dim):
        super(Generator, self).__init__()
        self.graph = graph
        self.num_relations = graph.relation_size
        self.num_layers = num_layers
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        # token ids: relations 0..|R|-1, END = |R|, PAD = |R| + 1 (generators.py:14-17)
        self.vocab_size = self.num_relations + 2
        self.label_size = self.num_relations + 1
        self.ending_idx = self.num_relations
        self.padding_idx = self.num_relations + 1
        self.embedding = torch.nn.Embedding(self.vocab_size, embedding_dim, padding_idx=self.padding_idx)
        self.rnn = torch.nn.LSTM(2 * embedding_dim, hidden_dim, num_layers, batch_first=True)
        self.linear = torch.nn.Linear(hidden_dim, self.label_size)
        self.criterion = torch.nn.CrossEntropyLoss(reduction="none")

    def forward(self, inputs, relation, hidden):
        """(N, T) tokens, (N,) head relations, (h0, c0) -> ((N, T, |R|+1) logits,
        (hT, cT)) (generators.py:23-29)."""
        x = self.embedding(inputs)
        head = self.embedding(relation).unsqueeze(1).expand_as(x)
        outputs, hidden = self.rnn(torch.cat([x, head], dim=-1), hidden)
        return self.linear(outputs), hidden

    def loss(self, inputs, target, mask, weight, hidden):
        """Weighted next-token cross entropy over the unpadded positions,
        Σ w_i·CE / Σ w_i with a rule's weight on each of its positions
        (generators.py:31-37).  On the CPU the unpadded positions are
        gathered in row-major order before the sums, as the reference does, so
        the fp32 sums round identically and a seeded run trains to bitwise the
        same weights (which sample() needs to draw the reference's rules).  On
        a GPU (whose reductions round differently from the CPU reference's in
        any case) the sums run densely with padded positions weighted 0: the
        same value without the gather's host sync."""
        logits, _ = self.forward(inputs, inputs[:, 0], hidden)
        if logits.is_cuda:
            # PAD (= label_size) is not a class: point padded targets at class 0, weight 0
            tgt = torch.where(mask, target, torch.zeros_like(target))
            ce = F.cross_entropy(logits.reshape(-1, self.label_size), tgt.reshape(-1), reduction="none")
            w = (mask.to(logits.dtype) * weight.to(logits.dtype).unsqueeze(1)).reshape(-1)
            return (ce * w).sum() / w.sum()
        keep = mask.reshape(-1).nonzero().squeeze(1)
        picked = logits.reshape(-1, self.label_size).index_select(0, keep)
        ce = F.cross_entropy(picked, target.reshape(-1).index_select(0, keep), reduction="none")
        w = (mask.to(weight.dtype) * weight.unsqueeze(1)).reshape(-1).index_select(0, keep)
        return (ce * w).sum() / w.sum()
