"""Optional Kubernetes actuator (``GPUMGR=k8s``).

The node-local :class:`~.controller.GpuManager` is the default actuator: it
replaces Kubernetes on one MI355X node.  Clusters that schedule MI355X pods
with Kubernetes can keep doing so: this actuator forwards the same four
calls the reconcile core makes (``list_namespaced_{deployment,job}``,
``patch_namespaced_{deployment,job}``) to the official client, exactly as
the reference does (``autoscaler/autoscaler.py:79-151``: in-cluster config,
``AppsV1Api`` / ``BatchV1Api``), and converts the client's ``ApiException``
into :class:`~.resources.ActuatorError` so the core's error contract is the
same for both actuators (a failed PATCH is logged and retried next tick, a
failed LIST is fatal).

The ``kubernetes`` package is not a dependency of this framework; it is
imported on first use, and a clear :class:`ActuatorError` (503) is raised
when it is missing.
"""
import logging

from .resources import ActuatorError

logger = logging.getLogger('KubernetesActuator')


def _load_client():
    try:
        import kubernetes  # noqa: F401
        from kubernetes import client, config
    except ImportError as err:
        raise ActuatorError(503, 'GPUMGR=k8s needs the `kubernetes` Python '
                                 'package (%s)' % err)
    return client, config


class KubernetesActuator(object):
    """Thin forwarding actuator over ``AppsV1Api`` / ``BatchV1Api``."""

    def __init__(self, in_cluster=True):
        client, config = _load_client()
        try:
            if in_cluster:
                config.load_incluster_config()
            else:
                config.load_kube_config()
        except Exception as err:  # config exceptions differ per version
            raise ActuatorError(503, 'cannot load Kubernetes config: %s'
                                % err)
        self._client = client
        self.apps = client.AppsV1Api()
        self.batch = client.BatchV1Api()

    def _call(self, func, *args):
        api_exception = getattr(getattr(self._client, 'rest', None),
                                'ApiException', None)
        try:
            return func(*args)
        except Exception as err:  # pylint: disable=broad-except
            if api_exception is not None and isinstance(err, api_exception):
                raise ActuatorError(getattr(err, 'status', 500),
                                    getattr(err, 'reason', str(err)),
                                    getattr(err, 'body', None))
            raise

    def list_namespaced_deployment(self, namespace):
        return self._call(self.apps.list_namespaced_deployment, namespace)

    def list_namespaced_job(self, namespace):
        return self._call(self.batch.list_namespaced_job, namespace)

    def patch_namespaced_deployment(self, name, namespace, body):
        return self._call(self.apps.patch_namespaced_deployment, name,
                          namespace, body)

    def patch_namespaced_job(self, name, namespace, body):
        return self._call(self.batch.patch_namespaced_job, name, namespace,
                          body)
