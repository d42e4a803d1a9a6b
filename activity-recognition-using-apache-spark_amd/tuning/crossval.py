"""ParamGridBuilder / CrossValidator / TrainValidationSplit.

Reference: ``ParamGridBuilder().addGrid(lr.regParam, [0.1,0.3,0.5]).addGrid(
lr.elasticNetParam, [0.0,0.1,0.2]).build()`` and ``CrossValidator(estimator,
estimatorParamMaps, evaluator, numFolds=5)`` (``Main/main.py:202-215``; DT/RF with
an empty grid ``:379-402, 560-583``).  SURVEY.md C18/C20/C22, N9, §3.5.

Spark fits the 5 x 9 = 45 (fold, param map) models one after another
(``parallelism=1``) — the most expensive entry point of the reference (129.9 s).
Here, for LogisticRegression, all 45 fits are ONE batched device optimization
(``LogisticRegression.fit_many``): each fold is a 0/1 row-weight vector over the
resident training matrix, so the two GEMMs of every objective evaluation cover
all 45 models at once.  DecisionTree / RandomForest grow the trees of all k folds
as one level-synchronous forest (fold masks multiply the bootstrap weights; split
candidates come from the whole CV input, labels never); other estimators fit per
(fold, map) on the device.

Note on the objective: in the reference the CV evaluator is whatever object was
last assigned to ``evaluator`` — ``RegressionEvaluator(metricName="mae")``
(``Main/main.py:175``) — so its model selection minimizes the MAE of class
indices.  Any evaluator can be passed here; ``main.py`` defaults to accuracy and
offers ``--cv-metric mae`` for behavioural parity.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.split import kfold_ids, split_ids
from ..ops import rng
from ..data.table import Column, Table
from ..models.base import Estimator, Model, dp_allreduce, dp_context, dp_rows, features_tensor, labels_tensor, \
    new_uid, num_label_classes, resolve_device


def _pname(p) -> str:
    return p if isinstance(p, str) else getattr(p, "name", str(p))


class ParamGridBuilder:
    def __init__(self):
        self._grid: Dict[str, List] = {}
        self._base: Dict[str, object] = {}

    def addGrid(self, param, values: Sequence):
        self._grid[_pname(param)] = list(values)
        return self

    def baseOn(self, *pairs, **kw):
        for k, v in pairs:
            self._base[_pname(k)] = v
        self._base.update(kw)
        return self

    def build(self) -> List[Dict]:
        keys = list(self._grid)
        maps = []
        for combo in itertools.product(*(self._grid[k] for k in keys)):
            m = dict(self._base)
            m.update(dict(zip(keys, combo)))
            maps.append(m)
        return maps or [dict(self._base)]


def _lr_margins(models, hm) -> torch.Tensor:
    """Raw predictions ``[n, N, K]`` of n logistic-regression models (binomial: ``[-m, m]``): one
    launch of the evaluation kernel in prediction mode on the GPU."""
    from ..ops.logreg import logreg_margins_native, native_classes_ok

    k = models[0].coefficientMatrix.shape[0]
    if hm.device.type == "cuda" and native_classes_ok(k):
        KP = 8 if k <= 8 else 16
        # one batched weight table [n, F+1, KP] (row F = intercepts) instead of one per model
        coef = torch.stack([m.coefficientMatrix for m in models]).to(hm.device)
        F = coef.shape[2]
        W = torch.zeros(len(models), F + 1, KP, device=hm.device)
        W[:, :F, :k] = coef.transpose(1, 2)
        W[:, F, :k] = torch.stack([m.interceptVector for m in models]).to(hm.device)
        m = logreg_margins_native(hm, W, k, len(models))[:, :, :k]
        return torch.cat([-m, m], dim=2) if models[0].binomial else m
    return torch.stack([mm.predict_raw(hm) for mm in models])


class CrossValidatorModel(Model):
    def __init__(self, bestModel, avgMetrics: List[float], bestIndex: int, subModels=None, uid=None):
        super().__init__(uid or new_uid("CrossValidatorModel"))
        self.bestModel, self.avgMetrics, self.bestIndex, self.subModels = bestModel, avgMetrics, bestIndex, subModels

    def transform(self, table: Table) -> Table:
        return self.bestModel.transform(table)

    def __getattr__(self, item):  # delegate predict_all / num_classes ... to the best model
        if item in ("bestModel", "__setstate__", "__getstate__"):
            raise AttributeError(item)
        return getattr(self.bestModel, item)

    def __str__(self):
        return self.uid


def _batched_predictions(models, raw: torch.Tensor) -> torch.Tensor:
    """Predicted classes of a stack of models' raw outputs ``raw`` [n, N, K], as each model's
    ``transform`` would give them: argmax of the probabilities, or of the probabilities scaled by
    the model's ``thresholds`` when it has them (Spark scores CV folds through
    ``model.transform``, which applies the thresholds; ``Main/main.py:209-215``)."""
    if all(getattr(m, "thresholds", None) is None for m in models):
        return torch.argmax(raw, dim=2)  # probabilities are monotone in the raw scores per row
    preds = []
    for m, r in zip(models, raw):
        preds.append(m._predict_from_probability(m.raw_to_probability(r)))
    return torch.stack(preds)


class CrossValidator(Estimator):
    def __init__(self, estimator=None, estimatorParamMaps: Optional[List[Dict]] = None, evaluator=None,
                 numFolds: int = 3, seed: int = 0, parallelism: int = 1, collectSubModels: bool = False):
        super().__init__(new_uid("CrossValidator"))
        self.estimator, self.estimatorParamMaps, self.evaluator = estimator, estimatorParamMaps or [{}], evaluator
        self.numFolds, self.seed, self.parallelism, self.collectSubModels = numFolds, seed, parallelism, collectSubModels

    def fit(self, table: Table) -> CrossValidatorModel:
        est, maps, ev, k = self.estimator, self.estimatorParamMaps, self.evaluator, self.numFolds
        n_rows = table.count()

        def fold_ids_on(dev):
            # the Philox fold assignment (data/split.py kfold_ids) on the device for the batched paths: the
            # host form (numpy Philox + an upload) was ~0.5 ms of an ~4 ms LR CrossValidator fit with the
            # GPU idle (profiles/r5/lr_grad_blocks.md); bitwise the same ids (tests/test_gpu_models.py)
            if dev.type == "cuda":
                return rng.device_buckets(self.seed, rng.STREAM_KFOLD, 0, n_rows, [1.0] * k, dev)
            return torch.as_tensor(kfold_ids(n_rows, k, self.seed), device=dev)

        metrics = np.zeros((len(maps), k), dtype=np.float64)
        from ..models.logreg import FitSpec, LogisticRegression

        batch_refit = False
        if isinstance(est, LogisticRegression):
            from ..features.hybrid import hybrid_features

            dev = resolve_device(est.device)
            hm = hybrid_features(table, est.featuresCol, dev)
            y = labels_tensor(table, est.labelCol, dev)
            K = num_label_classes(table, est.labelCol, dev)
            fold_t = fold_ids_on(dev)
            in_fold = fold_t[None, :] == torch.arange(k, device=dev)[:, None]  # [k, N]: ONE launch, not k
            train_w = (~in_fold).float()
            specs, index = [], []
            subs = [est.copy(pm) for pm in maps]  # (one copy per map: the fold specs and the refits share it)
            for mi, sub in enumerate(subs):
                for f in range(k):
                    specs.append(FitSpec(train_w[f], sub.regParam, sub.elasticNetParam))
                    index.append((mi, f))
            # the refit of every candidate on the full data rides along in the same batched solve
            # (one more model per param map): the final model is then the winner's full-data fit,
            # with no separate fit after the selection — the same model Spark's refit produces
            n_cv = len(specs)
            batch_refit = not est.weightCol and all(set(pm) <= {"regParam", "elasticNetParam"} for pm in maps)
            if batch_refit:
                for sub in subs:
                    specs.append(FitSpec(None, sub.regParam, sub.elasticNetParam))
            # maxIter / tol / family etc. may differ per map only through regParam/elasticNetParam
            base = subs[0] if maps else est
            lo, hi = dp_rows(hm.n_rows)  # data parallel: every fit on this rank's row shard
            if dp_context() is not None:
                specs = [FitSpec(None if s.row_weight is None else s.row_weight[lo:hi], s.regParam, s.elasticNetParam)
                         for s in specs]
            # deferred: the fold scoring below is enqueued behind the batched solve before the one host
            # sync (finalize), and the model objects are built while the GPU solves
            models_all, finalize = base.fit_many(hm.rows(lo, hi), y[lo:hi], specs, K, allreduce=dp_allreduce(),
                                                 deferred=True)
            models, refits = models_all[:n_cv], models_all[n_cv:]
            # every (map, fold) model scored on its validation fold in ONE batched pass
            raw = _lr_margins(models, hm)                                          # [n, N, K]
            pred = _batched_predictions(models, raw)
            mask = in_fold[torch.arange(len(index), device=dev) % k]  # fold of model i = i % k (no upload)
            vals = ev.evaluate_batched(y, pred, mask, K, raw, host=False)
            finalize()
            vals = vals.cpu().numpy() if torch.is_tensor(vals) else vals
            for (mi, f), v in zip(index, vals):
                metrics[mi, f] = v
        elif hasattr(est, "fit_folds") and not getattr(est, "weightCol", None):
            # trees: every fold's tree(s) in one lock-step build; NaiveBayes: fold masks as row weights
            dev = resolve_device(est.device)
            X, y, K = est._prep(table)
            fold_t = fold_ids_on(dev)
            masks = torch.stack([(fold_t != f).float() for f in range(k)])
            # trees on the reference encoding: the one-hot-aware path (same forests)
            hyb = est._hybrid(table, X.device) if hasattr(est, "_hybrid") else None
            for mi, pm in enumerate(maps):
                e = est.copy(pm)
                fms = e.fit_folds(X, y, K, masks, hybrid=hyb) if hyb is not None else e.fit_folds(X, y, K, masks)
                raws = [m.predict_raw(X) for m in fms]
                pred = _batched_predictions(fms, torch.stack(raws))
                vals = ev.evaluate_batched(y, pred, masks == 0, K, torch.stack(raws))
                metrics[mi, :] = vals
        else:
            fold = kfold_ids(n_rows, k, self.seed)
            for f in range(k):
                tr = table.take_rows(np.nonzero(fold != f)[0])
                va = table.take_rows(np.nonzero(fold == f)[0])
                for mi, pm in enumerate(maps):
                    m = est.copy(pm).fit(tr)
                    metrics[mi, f] = ev.evaluate(m.transform(va))
        avg = metrics.mean(axis=1)
        best = int(np.argmax(avg) if ev.isLargerBetter() else np.argmin(avg))
        if isinstance(est, LogisticRegression) and batch_refit:
            best_model = refits[best]
            best_model.uid = est.uid
        else:
            best_model = est.copy(maps[best]).fit(table)
        return CrossValidatorModel(best_model, avg.tolist(), best)


class TrainValidationSplitModel(CrossValidatorModel):
    pass


class TrainValidationSplit(Estimator):
    def __init__(self, estimator=None, estimatorParamMaps=None, evaluator=None, trainRatio: float = 0.75,
                 seed: int = 0):
        super().__init__(new_uid("TrainValidationSplit"))
        self.estimator, self.estimatorParamMaps, self.evaluator = estimator, estimatorParamMaps or [{}], evaluator
        self.trainRatio, self.seed = trainRatio, seed

    def fit(self, table: Table) -> TrainValidationSplitModel:
        ids = split_ids(table.count(), [self.trainRatio, 1 - self.trainRatio], self.seed)
        tr = table.take_rows(np.nonzero(ids == 0)[0])
        va = table.take_rows(np.nonzero(ids == 1)[0])
        mets = [self.evaluator.evaluate(self.estimator.copy(pm).fit(tr).transform(va)) for pm in
                self.estimatorParamMaps]
        best = int(np.argmax(mets) if self.evaluator.isLargerBetter() else np.argmin(mets))
        return TrainValidationSplitModel(self.estimator.copy(self.estimatorParamMaps[best]).fit(table), mets, best)
