"""placeholder, replaced below"""
class DistMatrix:  # noqa
    pass
def get_context():
    return None
