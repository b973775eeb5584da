"""Kubernetes-shaped resource records served by the node-local GPU manager.

The reference reads ``Deployment.spec.replicas``,
``Deployment.status.available_replicas`` and ``Job.spec.parallelism``
(``autoscaler/autoscaler.py:172-190``) and PATCHes ``{'spec': {'replicas':
n}}`` / ``{'spec': {'parallelism': n}}`` (``autoscaler.py:230-237``).  The GPU
manager exposes the same shape so the reconcile core keeps its logic:

* ``spec.replicas`` / ``spec.parallelism`` = declared worker count;
* ``status.ready_replicas`` = workers that published READY (weights in HBM
  + warm-start kernel done);
* ``status.available_replicas`` = READY workers in the last *fenced*
  membership (the set every GPU's process agreed on over the node
  communicator) -- what the reference's observer reads with
  ``only_running`` (``autoscaler.py:176-179``).  It lags READY by one fence
  (~1 ms) and stays behind while fencing fails; ``status.fence`` says why.
  Without fencing it equals ``ready_replicas``;
* ``status.active`` / ``status.succeeded`` / ``status.failed`` for jobs.
"""


class ActuatorError(Exception):
    """Failure of an actuation call (the ``kubernetes ApiException`` analog).

    ``status`` follows HTTP conventions (404 unknown resource, 409 conflict,
    422 invalid body, 503 manager unavailable)."""

    def __init__(self, status=500, reason='', body=None):
        Exception.__init__(self, '(%s) Reason: %s' % (status, reason))
        self.status = status
        self.reason = reason
        self.body = body


class _Bag(object):
    def __init__(self, **fields):
        self.__dict__.update(fields)

    def to_dict(self):
        return dict(self.__dict__)

    def __repr__(self):
        return '%s(%s)' % (type(self).__name__, ', '.join(
            '%s=%r' % kv for kv in sorted(self.__dict__.items())))

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__


class Metadata(_Bag):
    pass


class Spec(_Bag):
    pass


class Status(_Bag):
    pass


class ResourceView(_Bag):
    """Snapshot of one managed resource (``.metadata/.spec/.status``)."""

    @classmethod
    def build(cls, kind, namespace, name, declared, ready, active, succeeded=0,
              failed=0, generation=0, epoch=0, gpus=(), fenced=None,
              fence=None):
        metadata = Metadata(name=name, namespace=namespace,
                            generation=generation)
        available = ready if fenced is None else fenced
        if kind == 'deployment':
            spec = Spec(replicas=declared)
            status = Status(replicas=active, available_replicas=available,
                            ready_replicas=ready, fenced_replicas=available,
                            restarts=failed, fenced_epoch=epoch,
                            gpus=list(gpus), fence=dict(fence or {}))
        else:
            spec = Spec(parallelism=declared, completions=None)
            status = Status(active=active, ready=ready, succeeded=succeeded,
                            failed=failed, fenced_replicas=available,
                            fenced_epoch=epoch, gpus=list(gpus),
                            fence=dict(fence or {}))
        return cls(kind=kind, metadata=metadata, spec=spec, status=status)

    def to_dict(self):
        return {'kind': self.kind, 'metadata': self.metadata.to_dict(),
                'spec': self.spec.to_dict(), 'status': self.status.to_dict()}

    @classmethod
    def from_dict(cls, data):
        return cls(kind=data['kind'], metadata=Metadata(**data['metadata']),
                   spec=Spec(**data['spec']), status=Status(**data['status']))


class ResourceList(_Bag):
    """``.items`` container, the shape ``list_namespaced_*`` returns."""


def desired_from_body(kind, body):
    """Extract the replica count from a strategic-merge style body."""
    field = 'replicas' if kind == 'deployment' else 'parallelism'
    try:
        value = body['spec'][field]
    except (KeyError, TypeError):
        raise ActuatorError(422, 'body must carry spec.%s' % field, body)
    try:
        value = int(value)
    except (TypeError, ValueError):
        raise ActuatorError(422, 'spec.%s must be an integer' % field, body)
    if value < 0:
        raise ActuatorError(422, 'spec.%s must be >= 0' % field, body)
    return value
