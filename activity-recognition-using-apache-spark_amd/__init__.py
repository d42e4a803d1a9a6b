"""Source root of the ``har`` package (imported through ``har/__init__.py``).

Layout:

* ``data/``       columnar tables, CSV ingest + Spark-compatible schema inference,
                  Philox train/test split + k-fold, synthetic IMU streams
* ``features/``   StringIndexer / OneHotEncoder / VectorAssembler / Pipeline,
                  window featurization of raw accelerometer streams
* ``models/``     LogisticRegression, DecisionTree, RandomForest, NaiveBayes, MLP
* ``optim/``      batched device-resident L-BFGS / OWL-QN, fused Adam
* ``tuning/``     ParamGridBuilder, CrossValidator (all fold x param fits batched)
* ``evaluation/`` Binary / Multiclass / Regression evaluators (Spark definitions)
* ``ops/``        Python front-ends of the hand-written HIP/CDNA4 kernels
* ``parallel/``   one-process-per-GPU runtime over RCCL (``nccl`` backend) / gloo
* ``report/``     result.txt / metrics CSV / plots in the reference's formats
* ``utils/``      timers, tracing (roctx), persistence, checkpoints
"""
