"""Model and tokenizer converters to the `.m` / `.t` formats (reference: converter/*.py)."""
