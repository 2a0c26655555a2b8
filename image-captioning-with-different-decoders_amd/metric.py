"""Running-average metric (reference metric.py:29-46). Caption scoring
(get_eval_score: BLEU/METEOR/ROUGE/CIDEr, :7-27) is evaluation, outside the
training hot path this framework accelerates."""


class AccumulatingMetric():
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n

    def avg(self):
        if self.count == 0:
            return 0
        return self.sum / self.count


def get_eval_score(references, hypotheses):
    raise NotImplementedError("caption scoring (eval_func/*) is out of scope for the training path")
