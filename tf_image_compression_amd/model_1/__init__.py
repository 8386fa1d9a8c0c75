"""model_1 plugin module (reference: model_1/model.py)."""
