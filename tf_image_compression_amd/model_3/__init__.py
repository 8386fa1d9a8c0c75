"""model_3 plugin module (reference: model_3/model.py)."""
