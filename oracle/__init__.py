"""CPU oracle for the GPT-2 training step — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference semantics of the one hot path this repo
accelerates (forward -> loss -> backward -> grad collective -> clip-norm -> AdamW, plus the
loader's shard/batch indexing). It is the checker, never the thing measured or shipped:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
  import it;
* the product package ``gpt_2_distributed_amd`` never imports it and has no CPU fallback.

Parity pinning: the restatement is checked against golden vectors captured from the reference
itself (``/root/reference/model.py`` + ``dataloader.py`` imported in the build container by
``tests/golden/make_golden.py``), committed under ``tests/golden/``.

Modules
-------
model_ref   functional fp32 / bf16-autocast restatement of ``model.py`` (init, forward, per-op)
loader_ref  pure-python restatement of ``dataloader.py``'s shard/offset/batch order
train_ref   restatement of the ``train_gpt2_distributed.py:374-425`` step loop + AdamW math
"""
